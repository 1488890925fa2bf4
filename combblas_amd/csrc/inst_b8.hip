// inst_b8.hip -- instantiation of the SpGEMM/merge pipeline for value type uint8_t.
#include "spgemm_host.hpp"

cbg_status cbg_dispatch_b8(cbg_ctx* ctx, const cbg_dcsc_view* A, const cbg_dcsc_view* B, cbg_semiring sr,
                              uint32_t f, cbg_csc_result* C, int64_t* m) {
  return cbg::host::dispatch_sr<uint8_t, false>(ctx, A, B, sr, f, C, m);
}
cbg_status cbg_merge_b8(cbg_ctx* ctx, const cbg_csc_result* parts, int32_t k, cbg_semiring sr, uint32_t f,
                           cbg_csc_result* C) {
  return cbg::host::merge_impl<uint8_t>(ctx, parts, k, sr, f, C);
}
