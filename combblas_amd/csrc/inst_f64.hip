// inst_f64.hip -- instantiation of the SpGEMM/merge pipeline for value type double.
#include "spgemm_host.hpp"

cbg_status cbg_dispatch_f64(cbg_ctx* ctx, const cbg_dcsc_view* A, const cbg_dcsc_view* B, cbg_semiring sr,
                              uint32_t f, cbg_csc_result* C, int64_t* m) {
  return cbg::host::dispatch_sr<double, false>(ctx, A, B, sr, f, C, m);
}
cbg_status cbg_merge_f64(cbg_ctx* ctx, const cbg_csc_result* parts, int32_t k, cbg_semiring sr, uint32_t f,
                           cbg_csc_result* C) {
  return cbg::host::merge_impl<double>(ctx, parts, k, sr, f, C);
}

#ifdef CBG_STAMPS
extern "C" cbg_status cbg_debug_stamps(uint64_t* out, int reset) {
  unsigned long long h[32];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(cbg::g_stamps), sizeof(h)) != hipSuccess) return CBG_EDEVICE;
  for (int i = 0; i < 32; ++i) out[i] = h[i];
  if (reset) {
    memset(h, 0, sizeof(h));
    if (hipMemcpyToSymbol(HIP_SYMBOL(cbg::g_stamps), h, sizeof(h)) != hipSuccess) return CBG_EDEVICE;
  }
  return CBG_OK;
}
#endif
