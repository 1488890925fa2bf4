// cbgpu.hip -- C ABI (include/cbgpu.h) + host orchestration of the local SpGEMM on one MI355X.
//
// Pipeline per cbg_spgemm_local call (all on the context's stream):
//   stage inputs -> k_col_stats -> k_bin(symbolic) -> k_sym_{wave,block,window} -> scan -> alloc C
//   -> k_bin(numeric) -> k_num_{wave,block} -> k_window(numeric) for heavy + overflow columns.
// Two host synchronisations: class histograms (to size launches) and nnz(C) (to allocate C).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>
#include <memory>
#include "cbgpu.h"
#include "spgemm_kernels.hpp"

using namespace cbg;

#define HIPCHK(x)                                                                                   \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) {                                                                         \
      fprintf(stderr, "cbgpu: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
      return CBG_EDEVICE;                                                                           \
    }                                                                                               \
  } while (0)

namespace {

// symbolic classes: wave T = 64..1024 words, block T = 2048..32768 words, then window
constexpr int kSymWave = 5, kSymBlock = 5;
// numeric classes: wave T = 64..512 slots, block T = 1024..8192 slots, then window
constexpr int kNumWave = 4, kNumBlock = 4;
constexpr int kBlockNT = 512;
constexpr int kWinNT = 256;
constexpr int kMaxGrid = 4096;

struct DevBuf {
  void* p = nullptr;
  size_t n = 0;
  ~DevBuf() { if (p) (void)hipFree(p); }
  hipError_t reserve(size_t bytes) {
    if (bytes <= n) return hipSuccess;
    if (p) { (void)hipFree(p); p = nullptr; n = 0; }
    hipError_t e = hipMalloc(&p, bytes ? bytes : 16);
    if (e == hipSuccess) n = bytes;
    return e;
  }
  template <typename T> T* as() const { return (T*)p; }
};

size_t dt_size(cbg_dtype t) {
  switch (t) { case CBG_BOOL: return 1; case CBG_I32: case CBG_F32: return 4; default: return 8; }
}

template <typename V> struct DtOf;
template <> struct DtOf<double> { static constexpr cbg_dtype value = CBG_F64; };
template <> struct DtOf<float> { static constexpr cbg_dtype value = CBG_F32; };
template <> struct DtOf<int64_t> { static constexpr cbg_dtype value = CBG_I64; };
template <> struct DtOf<int32_t> { static constexpr cbg_dtype value = CBG_I32; };
template <> struct DtOf<uint8_t> { static constexpr cbg_dtype value = CBG_BOOL; };

struct Owner {                 // device storage behind a cbg_csc_result
  DevBuf cp, ir, val;
};

}  // namespace

struct cbg_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  hipEvent_t ev[8] = {};
  cbg_profile prof{};
  // workspace (grow-only)
  DevBuf flop, span, cnt, list, hist, cursor, scan_tiles, scalars, cur, nxt, ovf_list, stageA[5], stageB[5];
};

static hipError_t launch_cfg_lds(const void* fn, size_t lds) {
  if (lds > 64 * 1024) return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  return hipSuccess;
}

// ------------------------------------------------------------------------------- input staging
namespace {
template <typename V>
cbg_status stage(cbg_ctx* ctx, const cbg_dcsc_view* v, DevBuf* sb, DevCsc<V>* out) {
  const int pb = v->ptr_bytes ? v->ptr_bytes : v->idx_bytes;
  if ((v->idx_bytes != 4 && v->idx_bytes != 8) || (pb != 4 && pb != 8)) return CBG_EINVAL;
  if (v->nnz > 0 && (!v->cp || !v->ir)) return CBG_EINVAL;
  // a bool-typed operand of a non-bool product is a pattern (SelectMaxSRing<bool,T>, BoolCopy*)
  const bool pattern = !v->val || (v->val_type == CBG_BOOL && sizeof(V) != 1);
  if (!pattern && dt_size(v->val_type) != sizeof(V)) return CBG_EINVAL;
  if (v->nrow >= INT32_MAX) return CBG_EUNSUP;
  hipStream_t st = ctx->stream;
  const bool dcsc = v->jc != nullptr;
  const int64_t ncp = dcsc ? v->nzc + 1 : v->ncol + 1;
  out->nrow = v->nrow; out->ncol = v->ncol; out->nnz = v->nnz;
  const hipMemcpyKind kind = v->on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
  // colptr as int64 dense
  const int64_t* cp64 = nullptr;
  if (!dcsc && pb == 8 && v->on_device) {
    cp64 = (const int64_t*)v->cp;
  } else {
    HIPCHK(sb[0].reserve(sizeof(int64_t) * (v->ncol + 1)));
    // raw cp (and jc) to device first
    HIPCHK(sb[3].reserve(sizeof(int64_t) * (2 * ncp + 2)));
    int64_t* rawcp = sb[3].as<int64_t>();
    int64_t* rawjc = rawcp + ncp;
    HIPCHK(sb[2].reserve(sizeof(int32_t) * (2 * ncp + 2)));
    int32_t* t32 = sb[2].as<int32_t>();
    if (pb == 8) {
      HIPCHK(hipMemcpyAsync(rawcp, v->cp, sizeof(int64_t) * ncp, kind, st));
    } else {
      HIPCHK(hipMemcpyAsync(t32, v->cp, sizeof(int32_t) * ncp, kind, st));
      k_i32_to_i64<<<256, 256, 0, st>>>(ncp, t32, rawcp);
    }
    if (dcsc) {
      if (v->idx_bytes == 8) {
        HIPCHK(hipMemcpyAsync(rawjc, v->jc, sizeof(int64_t) * v->nzc, kind, st));
      } else {
        HIPCHK(hipMemcpyAsync(t32 + ncp, v->jc, sizeof(int32_t) * v->nzc, kind, st));
        k_i32_to_i64<<<256, 256, 0, st>>>(v->nzc, t32 + ncp, rawjc);
      }
    }
    if (dcsc) {
      const int64_t g = std::min<int64_t>((v->ncol + 256) / 256, kMaxGrid);
      k_dcsc_to_csc<<<(int)g, 256, 0, st>>>(v->ncol, v->nzc, rawcp, rawjc, sb[0].as<int64_t>());
    } else {
      HIPCHK(hipMemcpyAsync(sb[0].p, rawcp, sizeof(int64_t) * (v->ncol + 1), hipMemcpyDeviceToDevice, st));
    }
    cp64 = sb[0].as<int64_t>();
  }
  out->cp = cp64;
  // row indices as int32
  if (v->idx_bytes == 4 && v->on_device) {
    out->ir = (const int32_t*)v->ir;
  } else {
    HIPCHK(sb[1].reserve(sizeof(int32_t) * (v->nnz + 1)));
    if (v->idx_bytes == 4) {
      HIPCHK(hipMemcpyAsync(sb[1].p, v->ir, sizeof(int32_t) * v->nnz, kind, st));
    } else {
      HIPCHK(sb[4].reserve(sizeof(int64_t) * (v->nnz + 1)));
      HIPCHK(hipMemcpyAsync(sb[4].p, v->ir, sizeof(int64_t) * v->nnz, kind, st));
      k_widen_idx<<<1024, 256, 0, st>>>(v->nnz, sb[4].as<int64_t>(), sb[1].as<int32_t>());
      HIPCHK(hipStreamSynchronize(st));   // sb[4] is reused for values below
    }
    out->ir = sb[1].as<int32_t>();
  }
  // values
  if (pattern || v->nnz == 0) {
    out->val = nullptr;
  } else if (v->on_device) {
    out->val = (const V*)v->val;
  } else {
    HIPCHK(sb[4].reserve(sizeof(V) * (size_t)(v->nnz + 1)));
    HIPCHK(hipMemcpyAsync(sb[4].p, v->val, sizeof(V) * v->nnz, hipMemcpyHostToDevice, st));
    out->val = sb[4].as<V>();
  }
  return CBG_OK;
}

inline int64_t grid_for(int64_t items, int64_t per_block, int64_t cap) {
  return std::max<int64_t>(1, std::min<int64_t>((items + per_block - 1) / per_block, cap));
}

struct Classes {
  std::vector<unsigned long long> hist;   // per class counts
  std::vector<unsigned long long> off;    // exclusive offsets
};

cbg_status bin_columns(cbg_ctx* ctx, int64_t ncol, const int64_t* cnt, const int2* span, BinParams bp,
                       int32_t* list, Classes* cl) {
  hipStream_t st = ctx->stream;
  const int ncls = bp.nwave + bp.nblock + 2;
  HIPCHK(ctx->hist.reserve(sizeof(unsigned long long) * 64));
  unsigned long long* hist = ctx->hist.as<unsigned long long>();
  unsigned long long* cursor = hist + 32;
  HIPCHK(hipMemsetAsync(hist, 0, sizeof(unsigned long long) * 64, st));
  const int64_t g = (ncol + 255) / 256;
  k_bin<<<(int)g, 256, 0, st>>>(ncol, cnt, span, bp, 0, hist, cursor, list);
  cl->hist.assign(ncls, 0);
  HIPCHK(hipMemcpyAsync(cl->hist.data(), hist, sizeof(unsigned long long) * ncls, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  cl->off.assign(ncls + 1, 0);
  for (int c = 0; c < ncls; ++c) cl->off[c + 1] = cl->off[c] + cl->hist[c];
  HIPCHK(hipMemcpyAsync(cursor, cl->off.data(), sizeof(unsigned long long) * ncls, hipMemcpyHostToDevice, st));
  k_bin<<<(int)g, 256, 0, st>>>(ncol, cnt, span, bp, 1, hist, cursor, list);
  return CBG_OK;
}

// ------------------------------------------------------------------------------- symbolic launch
template <int LOGT>
void launch_sym_wave(hipStream_t st, const int32_t* l, int64_t n, const DevCsc<int32_t>& A, const int64_t* Bcp,
                     const int32_t* Bir, const int2* span, int64_t* nnz) {
  k_sym_wave<LOGT><<<(int)grid_for(n, 4, kMaxGrid * 2), 256, 0, st>>>(l, n, A.cp, A.ir, Bcp, Bir, span, nnz);
}
template <int LOGT>
hipError_t launch_sym_block(hipStream_t st, const int32_t* l, int64_t n, const int64_t* Acp, const int32_t* Air,
                            const int64_t* Bcp, const int32_t* Bir, const int2* span, int64_t* nnz) {
  const size_t lds = (size_t)(1 << LOGT) * 4 + kBlockNT * 4 + 64;
  hipError_t e = launch_cfg_lds((const void*)k_sym_block<LOGT, kBlockNT>, lds);
  if (e != hipSuccess) return e;
  k_sym_block<LOGT, kBlockNT><<<(int)grid_for(n, 1, kMaxGrid), kBlockNT, lds, st>>>(l, n, Acp, Air, Bcp, Bir, span, nnz);
  return hipGetLastError();
}

template <int LOGT, class SRT, typename V>
void launch_num_wave(hipStream_t st, const int32_t* l, int64_t n, const DevCsc<V>& A, const DevCsc<V>& B,
                     const int2* span, const NumOut<V>& o) {
  k_num_wave<SRT, V, LOGT><<<(int)grid_for(n, 4, kMaxGrid * 2), 256, 0, st>>>(l, n, A, B, span, o);
}
template <int LOGT, class SRT, typename V>
hipError_t launch_num_block(hipStream_t st, const int32_t* l, int64_t n, const DevCsc<V>& A, const DevCsc<V>& B,
                            const int2* span, const NumOut<V>& o) {
  using Acc = typename SRT::Acc;
  const size_t TC = (size_t)(1 << LOGT) + kBlockNT;
  const size_t lds = TC * (sizeof(Acc) + 4) + kBlockNT * 4 + 64;
  hipError_t e = launch_cfg_lds((const void*)k_num_block<SRT, V, LOGT, kBlockNT>, lds);
  if (e != hipSuccess) return e;
  k_num_block<SRT, V, LOGT, kBlockNT><<<(int)grid_for(n, 1, kMaxGrid), kBlockNT, lds, st>>>(l, n, A, B, span, o);
  return hipGetLastError();
}
template <int MODE, class SRT, typename V, int W>
hipError_t launch_window(hipStream_t st, const int32_t* l, const int* count_dev, int64_t count_host, int64_t grid,
                         const DevCsc<V>& A, const DevCsc<V>& B, const int2* span, int64_t* cur, int32_t* nxt,
                         int64_t* nnz, const NumOut<V>& o) {
  using Acc = typename SRT::Acc;
  const size_t lds = (MODE == 1 ? (size_t)W * sizeof(Acc) : 0) + (size_t)(W / 32) * 4 + kWinNT * 4 + 64;
  hipError_t e = launch_cfg_lds((const void*)k_window<MODE, SRT, V, kWinNT, W>, lds);
  if (e != hipSuccess) return e;
  k_window<MODE, SRT, V, kWinNT, W><<<(int)grid, kWinNT, lds, st>>>(l, count_dev, count_host, A, B, span, cur, nxt, nnz, o);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------- the product
template <int SRI, typename V>
cbg_status spgemm_impl(cbg_ctx* ctx, const cbg_dcsc_view* Av, const cbg_dcsc_view* Bv, uint32_t flags,
                       cbg_csc_result* C, int64_t* mult_out) {
  using SRT = Semiring<SRI, V>;
  hipStream_t st = ctx->stream;
  cbg_profile& pf = ctx->prof;
  memset(&pf, 0, sizeof(pf));
  if (Av->ncol != Bv->nrow) return CBG_EDIM;
  const int64_t M = Av->nrow, N = Bv->ncol;

  std::unique_ptr<Owner> own(new Owner);
  memset(C, 0, sizeof(*C));
  C->nrow = M; C->ncol = N;
  C->val_type = DtOf<V>::value;
  HIPCHK(own->cp.reserve(sizeof(int64_t) * (N + 1)));
  int64_t* colptr = own->cp.as<int64_t>();

  HIPCHK(hipEventRecord(ctx->ev[0], st));
  if (Av->nnz == 0 || Bv->nnz == 0 || M == 0 || N == 0) {   // mtSpGEMM.h:478-481
    HIPCHK(hipMemsetAsync(colptr, 0, sizeof(int64_t) * (N + 1), st));
    HIPCHK(own->ir.reserve(4)); HIPCHK(own->val.reserve(8));
    C->colptr = colptr; C->row = own->ir.as<int32_t>(); C->val = own->val.p; C->nnz = 0;
    C->_owner = own.release();
    if (mult_out) *mult_out = 0;
    HIPCHK(hipStreamSynchronize(st));
    return CBG_OK;
  }
  DevCsc<V> A, B;
  cbg_status s;
  if ((s = stage<V>(ctx, Av, ctx->stageA, &A)) != CBG_OK) return s;
  if ((s = stage<V>(ctx, Bv, ctx->stageB, &B)) != CBG_OK) return s;

  // 1. column statistics
  HIPCHK(ctx->flop.reserve(sizeof(int64_t) * (N + 1)));
  HIPCHK(ctx->span.reserve(sizeof(int2) * (N + 1)));
  HIPCHK(ctx->cnt.reserve(sizeof(int64_t) * (N + 1)));
  HIPCHK(ctx->list.reserve(sizeof(int32_t) * (N + 1)));
  HIPCHK(ctx->scalars.reserve(64));
  HIPCHK(ctx->cur.reserve(sizeof(int64_t) * (B.nnz + 1)));
  HIPCHK(ctx->nxt.reserve(sizeof(int32_t) * (B.nnz + 1)));
  HIPCHK(ctx->ovf_list.reserve(sizeof(int32_t) * (N + 1)));
  int64_t* flop = ctx->flop.as<int64_t>();
  int2* span = ctx->span.as<int2>();
  int64_t* nnz = ctx->cnt.as<int64_t>();
  int32_t* list = ctx->list.as<int32_t>();
  unsigned long long* sc = ctx->scalars.as<unsigned long long>();   // [0] mults, [1] nnzC, [2] adderr|ovf
  int* adderr = (int*)(sc + 2);
  int* ovf_n = adderr + 1;
  HIPCHK(hipMemsetAsync(sc, 0, 64, st));
  HIPCHK(hipMemsetAsync(nnz, 0, sizeof(int64_t) * N, st));
  k_col_stats<V><<<(int)((N * 16 + 255) / 256), 256, 0, st>>>(N, A.cp, A.ir, B.cp, B.ir, flop, span, sc);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(ctx->ev[1], st));

  // 2. symbolic binning + kernels
  Classes cs;
  BinParams sbp{kSymWave, kSymBlock, 64, 1};
  if ((s = bin_columns(ctx, N, flop, span, sbp, list, &cs)) != CBG_OK) return s;
  HIPCHK(hipEventRecord(ctx->ev[2], st));
  {
    auto L = [&](int c) { return list + cs.off[c]; };
    auto n = [&](int c) { return (int64_t)cs.hist[c]; };
    DevCsc<int32_t> Ai{A.nrow, A.ncol, A.nnz, A.cp, A.ir, nullptr};
    if (n(1)) launch_sym_wave<6>(st, L(1), n(1), Ai, B.cp, B.ir, span, nnz);
    if (n(2)) launch_sym_wave<7>(st, L(2), n(2), Ai, B.cp, B.ir, span, nnz);
    if (n(3)) launch_sym_wave<8>(st, L(3), n(3), Ai, B.cp, B.ir, span, nnz);
    if (n(4)) launch_sym_wave<9>(st, L(4), n(4), Ai, B.cp, B.ir, span, nnz);
    if (n(5)) launch_sym_wave<10>(st, L(5), n(5), Ai, B.cp, B.ir, span, nnz);
    hipError_t e = hipSuccess;
    if (n(6) && e == hipSuccess) e = launch_sym_block<11>(st, L(6), n(6), A.cp, A.ir, B.cp, B.ir, span, nnz);
    if (n(7) && e == hipSuccess) e = launch_sym_block<12>(st, L(7), n(7), A.cp, A.ir, B.cp, B.ir, span, nnz);
    if (n(8) && e == hipSuccess) e = launch_sym_block<13>(st, L(8), n(8), A.cp, A.ir, B.cp, B.ir, span, nnz);
    if (n(9) && e == hipSuccess) e = launch_sym_block<14>(st, L(9), n(9), A.cp, A.ir, B.cp, B.ir, span, nnz);
    if (n(10) && e == hipSuccess) e = launch_sym_block<15>(st, L(10), n(10), A.cp, A.ir, B.cp, B.ir, span, nnz);
    if (n(11) && e == hipSuccess) {
      NumOut<V> dummy{};
      e = launch_window<0, SRT, V, kSymWinRows>(st, L(11), nullptr, n(11), grid_for(n(11), 1, 1024), A, B, span,
                                                ctx->cur.as<int64_t>(), ctx->nxt.as<int32_t>(), nnz, dummy);
    }
    if (e != hipSuccess) { fprintf(stderr, "cbgpu: symbolic launch: %s\n", hipGetErrorString(e)); return CBG_EDEVICE; }
    HIPCHK(hipGetLastError());
  }
  HIPCHK(hipEventRecord(ctx->ev[3], st));

  // 3. scan -> colptr, nnz(C)
  const int64_t ntiles = (N + kScanTile - 1) / kScanTile;
  HIPCHK(ctx->scan_tiles.reserve(sizeof(int64_t) * (ntiles + 1)));
  k_scan_tiles<<<(int)ntiles, 256, 0, st>>>(N, nnz, ctx->scan_tiles.as<int64_t>());
  k_scan_sums<<<1, 1024, 0, st>>>(ntiles, ctx->scan_tiles.as<int64_t>(), (int64_t*)(sc + 1));
  k_scan_apply<<<(int)ntiles, 256, 0, st>>>(N, nnz, ctx->scan_tiles.as<int64_t>(), colptr);
  HIPCHK(hipGetLastError());
  unsigned long long hsc[2];
  HIPCHK(hipMemcpyAsync(hsc, sc, 16, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  HIPCHK(hipEventRecord(ctx->ev[4], st));
  const int64_t mults = (int64_t)hsc[0], nnzc = (int64_t)hsc[1];
  pf.multiplies = mults; pf.nnz_out = nnzc;
  HIPCHK(own->ir.reserve(sizeof(int32_t) * (nnzc + 1)));
  HIPCHK(own->val.reserve(sizeof(V) * (nnzc + 1)));

  // 4. numeric binning + kernels
  Classes cn;
  BinParams nbp{kNumWave, kNumBlock, 64, 0};
  if ((s = bin_columns(ctx, N, nnz, span, nbp, list, &cn)) != CBG_OK) return s;
  for (int c = 0; c < (int)cn.hist.size() && c < 16; ++c) pf.bins[c] = (int64_t)cn.hist[c];
  NumOut<V> o{colptr, own->ir.as<int32_t>(), own->val.as<V>(), adderr, ovf_n, ctx->ovf_list.as<int32_t>()};
  {
    auto L = [&](int c) { return list + cn.off[c]; };
    auto n = [&](int c) { return (int64_t)cn.hist[c]; };
    if (n(1)) launch_num_wave<6, SRT, V>(st, L(1), n(1), A, B, span, o);
    if (n(2)) launch_num_wave<7, SRT, V>(st, L(2), n(2), A, B, span, o);
    if (n(3)) launch_num_wave<8, SRT, V>(st, L(3), n(3), A, B, span, o);
    if (n(4)) launch_num_wave<9, SRT, V>(st, L(4), n(4), A, B, span, o);
    hipError_t e = hipSuccess;
    if (n(5) && e == hipSuccess) e = launch_num_block<10, SRT, V>(st, L(5), n(5), A, B, span, o);
    if (n(6) && e == hipSuccess) e = launch_num_block<11, SRT, V>(st, L(6), n(6), A, B, span, o);
    if (n(7) && e == hipSuccess) e = launch_num_block<12, SRT, V>(st, L(7), n(7), A, B, span, o);
    if (n(8) && e == hipSuccess) e = launch_num_block<13, SRT, V>(st, L(8), n(8), A, B, span, o);
    if (n(9) && e == hipSuccess)
      e = launch_window<1, SRT, V, kWinRows>(st, L(9), nullptr, n(9), grid_for(n(9), 1, 2048), A, B, span,
                                             ctx->cur.as<int64_t>(), ctx->nxt.as<int32_t>(), nnz, o);
    // overflow fallback: columns whose order-preserving hash ran past its tail
    if (e == hipSuccess)
      e = launch_window<1, SRT, V, kWinRows>(st, ctx->ovf_list.as<int32_t>(), ovf_n, 0, 512, A, B, span,
                                             ctx->cur.as<int64_t>(), ctx->nxt.as<int32_t>(), nnz, o);
    if (e != hipSuccess) { fprintf(stderr, "cbgpu: numeric launch: %s\n", hipGetErrorString(e)); return CBG_EDEVICE; }
    HIPCHK(hipGetLastError());
  }
  HIPCHK(hipEventRecord(ctx->ev[5], st));
  int herr[2];
  HIPCHK(hipMemcpyAsync(herr, adderr, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  float t;
  (void)hipEventElapsedTime(&t, ctx->ev[0], ctx->ev[1]); pf.flops_ms = t;
  (void)hipEventElapsedTime(&t, ctx->ev[1], ctx->ev[2]); pf.bin_ms = t;
  (void)hipEventElapsedTime(&t, ctx->ev[2], ctx->ev[3]); pf.symbolic_ms = t;
  (void)hipEventElapsedTime(&t, ctx->ev[3], ctx->ev[4]); pf.scan_ms = t;
  (void)hipEventElapsedTime(&t, ctx->ev[4], ctx->ev[5]); pf.numeric_ms = t;
  (void)hipEventElapsedTime(&t, ctx->ev[0], ctx->ev[5]); pf.total_ms = t;
  pf.bins[15] = herr[1];   // overflow-fallback columns
  C->nnz = nnzc;
  C->colptr = colptr;
  C->row = own->ir.as<int32_t>();
  C->val = own->val.p;
  C->multiplies = mults;
  C->_owner = own.release();
  if (mult_out) *mult_out = mults;
  if (herr[0]) return CBG_EADD;
  return CBG_OK;
}

template <typename V>
cbg_status dispatch_sr(cbg_ctx* ctx, const cbg_dcsc_view* A, const cbg_dcsc_view* B, cbg_semiring sr, uint32_t f,
                       cbg_csc_result* C, int64_t* m) {
  switch (sr) {
    case CBG_SR_PLUS_TIMES: return spgemm_impl<SR_PLUS_TIMES, V>(ctx, A, B, f, C, m);
    case CBG_SR_MIN_PLUS: return spgemm_impl<SR_MIN_PLUS, V>(ctx, A, B, f, C, m);
    case CBG_SR_SELECT2ND: return spgemm_impl<SR_SELECT2ND, V>(ctx, A, B, f, C, m);
    case CBG_SR_SELECT_MAX: return spgemm_impl<SR_SELECT_MAX, V>(ctx, A, B, f, C, m);
    case CBG_SR_SELECT_MAX_BOOL: return spgemm_impl<SR_SELECT_MAX_BOOL, V>(ctx, A, B, f, C, m);
    case CBG_SR_BOOL_COPY1ST: return spgemm_impl<SR_BOOL_COPY1ST, V>(ctx, A, B, f, C, m);
    case CBG_SR_BOOL_COPY2ND: return spgemm_impl<SR_BOOL_COPY2ND, V>(ctx, A, B, f, C, m);
  }
  return CBG_EUNSUP;
}

}  // namespace

// =============================================================================== C ABI
extern "C" {

int32_t cbg_abi_version(void) { return CBG_ABI_VERSION; }

const char* cbg_strerror(cbg_status s) {
  switch (s) {
    case CBG_OK: return "ok";
    case CBG_EDIM: return "dimension mismatch (DIMMISMATCH 3002)";
    case CBG_EALIAS: return "matrix alias (MATRIXALIAS 3005)";
    case CBG_ENOMEM: return "out of device memory";
    case CBG_EUNSUP: return "unsupported semiring/dtype";
    case CBG_EDEVICE: return "HIP device error or no GPU";
    case CBG_EADD: return "semiring add() called on BoolCopy1st/2nd (reference throws)";
    case CBG_EINVAL: return "invalid matrix view";
    case CBG_ECOMM: return "RCCL communication error";
  }
  return "unknown status";
}

cbg_status cbg_init(int device, cbg_ctx** out) {
  if (!out) return CBG_EINVAL;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= device || device < 0) return CBG_EDEVICE;
  HIPCHK(hipSetDevice(device));
  cbg_ctx* c = new cbg_ctx;
  c->device = device;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) { delete c; return CBG_EDEVICE; }
  c->own_stream = true;
  for (auto& e : c->ev)
    if (hipEventCreate(&e) != hipSuccess) { delete c; return CBG_EDEVICE; }
  *out = c;
  return CBG_OK;
}

cbg_status cbg_destroy(cbg_ctx* c) {
  if (!c) return CBG_OK;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  for (auto& e : c->ev) if (e) (void)hipEventDestroy(e);
  if (c->own_stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return CBG_OK;
}

cbg_status cbg_set_stream(cbg_ctx* c, void* s) {
  if (!c) return CBG_EINVAL;
  if (c->own_stream) { (void)hipStreamSynchronize(c->stream); (void)hipStreamDestroy(c->stream); }
  if (s) { c->stream = (hipStream_t)s; c->own_stream = false; }
  else { HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)); c->own_stream = true; }
  return CBG_OK;
}

cbg_status cbg_synchronize(cbg_ctx* c) {
  if (!c) return CBG_EINVAL;
  HIPCHK(hipStreamSynchronize(c->stream));
  return CBG_OK;
}

cbg_status cbg_spgemm_local(cbg_ctx* ctx, const cbg_dcsc_view* A, const cbg_dcsc_view* B, cbg_semiring sr,
                            cbg_dtype out_type, uint32_t flags, cbg_csc_result* C, int64_t* multiplies_out) {
  if (!ctx || !A || !B || !C) return CBG_EINVAL;
  HIPCHK(hipSetDevice(ctx->device));
  switch (out_type) {
    case CBG_F64: return dispatch_sr<double>(ctx, A, B, sr, flags, C, multiplies_out);
    case CBG_F32: return dispatch_sr<float>(ctx, A, B, sr, flags, C, multiplies_out);
    case CBG_I64: return dispatch_sr<int64_t>(ctx, A, B, sr, flags, C, multiplies_out);
    case CBG_I32: return dispatch_sr<int32_t>(ctx, A, B, sr, flags, C, multiplies_out);
    case CBG_BOOL: return dispatch_sr<uint8_t>(ctx, A, B, sr, flags, C, multiplies_out);
  }
  return CBG_EUNSUP;
}

cbg_status cbg_estimate(cbg_ctx* ctx, const cbg_dcsc_view* A, const cbg_dcsc_view* B, int64_t* mults,
                        int64_t* nnzc) {
  // symbolic == the first half of the product; run the pattern product and read its size
  cbg_dcsc_view a = *A, b = *B;
  a.val = nullptr; b.val = nullptr;
  a.val_type = b.val_type = CBG_BOOL;
  cbg_csc_result C;
  cbg_status s = cbg_spgemm_local(ctx, &a, &b, CBG_SR_PLUS_TIMES, CBG_BOOL, 0, &C, mults);
  if (s != CBG_OK) return s;
  if (nnzc) *nnzc = C.nnz;
  cbg_result_free(ctx, &C);
  return CBG_OK;
}

cbg_status cbg_result_to_host(cbg_ctx* ctx, const cbg_csc_result* C, int64_t* colptr, int32_t* row, void* val) {
  if (!ctx || !C) return CBG_EINVAL;
  HIPCHK(hipSetDevice(ctx->device));
  if (colptr) HIPCHK(hipMemcpyAsync(colptr, C->colptr, sizeof(int64_t) * (C->ncol + 1), hipMemcpyDeviceToHost, ctx->stream));
  if (row && C->nnz) HIPCHK(hipMemcpyAsync(row, C->row, sizeof(int32_t) * C->nnz, hipMemcpyDeviceToHost, ctx->stream));
  if (val && C->nnz) HIPCHK(hipMemcpyAsync(val, C->val, dt_size(C->val_type) * C->nnz, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return CBG_OK;
}

void cbg_result_free(cbg_ctx* ctx, cbg_csc_result* C) {
  if (!C) return;
  if (ctx) { (void)hipSetDevice(ctx->device); (void)hipStreamSynchronize(ctx->stream); }
  delete (Owner*)C->_owner;
  memset(C, 0, sizeof(*C));
}

cbg_status cbg_upload(cbg_ctx* ctx, const cbg_dcsc_view* v, cbg_csc_result* out) {
  if (!ctx || !v || !out) return CBG_EINVAL;
  const int pb = v->ptr_bytes ? v->ptr_bytes : v->idx_bytes;
  if (v->jc || (v->idx_bytes != 8 && v->idx_bytes != 4) || (pb != 8 && pb != 4)) return CBG_EINVAL;
  HIPCHK(hipSetDevice(ctx->device));
  std::unique_ptr<Owner> own(new Owner);
  hipStream_t st = ctx->stream;
  const hipMemcpyKind kind = v->on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
  HIPCHK(own->cp.reserve(8 * (v->ncol + 1)));
  HIPCHK(own->ir.reserve(4 * (v->nnz + 1)));
  const size_t vs = v->val ? dt_size(v->val_type) : 0;
  HIPCHK(own->val.reserve(vs * (v->nnz + 1) + 8));
  DevBuf tmp;
  DevBuf tmp2;
  if (pb == 8) {
    HIPCHK(hipMemcpyAsync(own->cp.p, v->cp, 8 * (v->ncol + 1), kind, st));
  } else {
    HIPCHK(tmp2.reserve(4 * (v->ncol + 2)));
    HIPCHK(hipMemcpyAsync(tmp2.p, v->cp, 4 * (v->ncol + 1), kind, st));
    k_i32_to_i64<<<256, 256, 0, st>>>(v->ncol + 1, tmp2.as<int32_t>(), own->cp.as<int64_t>());
  }
  if (v->idx_bytes == 8) {
    HIPCHK(tmp.reserve(8 * (v->nnz + 1)));
    HIPCHK(hipMemcpyAsync(tmp.p, v->ir, 8 * v->nnz, kind, st));
    k_widen_idx<<<1024, 256, 0, st>>>(v->nnz, tmp.as<int64_t>(), own->ir.as<int32_t>());
  } else {
    HIPCHK(hipMemcpyAsync(own->ir.p, v->ir, 4 * v->nnz, kind, st));
  }
  if (v->val && v->nnz) HIPCHK(hipMemcpyAsync(own->val.p, v->val, vs * v->nnz, kind, st));
  HIPCHK(hipStreamSynchronize(st));
  memset(out, 0, sizeof(*out));
  out->nrow = v->nrow; out->ncol = v->ncol; out->nnz = v->nnz;
  out->colptr = own->cp.as<int64_t>(); out->row = own->ir.as<int32_t>();
  out->val = v->val ? own->val.p : nullptr;
  out->val_type = v->val_type;
  out->_owner = own.release();
  return CBG_OK;
}

cbg_status cbg_result_view(const cbg_csc_result* C, cbg_dcsc_view* v) {
  if (!C || !v) return CBG_EINVAL;
  memset(v, 0, sizeof(*v));
  v->nrow = C->nrow; v->ncol = C->ncol; v->nnz = C->nnz; v->nzc = C->ncol;
  v->cp = C->colptr; v->jc = nullptr; v->ir = C->row; v->idx_bytes = 4; v->ptr_bytes = 8;
  v->val = C->val; v->val_type = C->val_type; v->on_device = 1;
  return CBG_OK;
}

cbg_status cbg_last_profile(cbg_ctx* ctx, cbg_profile* p) {
  if (!ctx || !p) return CBG_EINVAL;
  *p = ctx->prof;
  return CBG_OK;
}

}  // extern "C"

extern "C" cbg_status cbg_generate_rmat(cbg_ctx* ctx, int32_t scale, int32_t edgefactor, uint64_t seed,
                                        cbg_csc_result* A) {
  if (!ctx || !A) return CBG_EINVAL;
  cbg_host_csc h;
  cbg_status s = cbg_rmat_host(scale, edgefactor, seed, &h);
  if (s != CBG_OK) return s;
  cbg_dcsc_view v{};
  v.nrow = h.nrow; v.ncol = h.ncol; v.nnz = h.nnz; v.nzc = h.ncol;
  v.cp = h.colptr; v.ir = h.row; v.idx_bytes = 4; v.ptr_bytes = 8;
  v.val = h.val; v.val_type = CBG_F64; v.on_device = 0;
  s = cbg_upload(ctx, &v, A);
  cbg_host_free(&h);
  return s;
}

extern "C" cbg_status cbg_merge(cbg_ctx* ctx, const cbg_csc_result* parts, int32_t nparts, cbg_semiring sr,
                                cbg_dtype val_type, uint32_t flags, cbg_csc_result* C) {
  (void)ctx; (void)parts; (void)nparts; (void)sr; (void)val_type; (void)flags; (void)C;
  return CBG_EUNSUP;   // device multiway merge: see DESIGN.md (next milestone)
}
