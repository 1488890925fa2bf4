#pragma once
// spgemm_host.hpp -- host orchestration of the local SpGEMM on one MI355X (templates + workspace).
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
#include <map>
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

#define CBGCHK(x)                \
  do {                           \
    cbg_status s_ = (x);         \
    if (s_ != CBG_OK) return s_; \
  } while (0)

// refuse a phase's launches when a workspace buffer it captured was reallocated since (Captures)
#define CAPCHK(c)                                                                                            \
  do {                                                                                                       \
    const char* w_ = "?";                                                                                    \
    if (!(c).ok(&w_)) {                                                                                      \
      fprintf(stderr, "cbgpu: workspace '%s' reallocated after its pointer was taken (%s:%d)\n", w_, __FILE__, \
              __LINE__);                                                                                     \
      return CBG_EINVAL;                                                                                     \
    }                                                                                                        \
  } while (0)

namespace cbg { namespace host {

// symbolic classes: wave T = 64..1024 words, block T = 2048..32768 words, then window
constexpr int kSymWave = 5, kSymBlock = 5;
// numeric classes: wave T = 64..512 slots, block T = 1024..8192 slots, then window
constexpr int kNumWave = 4, kNumBlock = 4;
constexpr int kBlockNT = 512;
constexpr int kWinNT = 256;
constexpr int kMaxGrid = 4096;
#ifndef CBG_KNOWN_SORT_DEFAULT
#define CBG_KNOWN_SORT_DEFAULT 1   // rows-known units in first-subwindow order (CBG_KNOWN_SORT=0 at run time: list order); s20 heavy 30.3 -> 29.9 ms, s21 96.6 -> 94.9 ms, profiles/r05p_known_sort_ab.txt
#endif
constexpr int64_t kSymPartGrid = kMaxGrid * 2;   // k_sym_part's largest grid (HeavyOut::chunk slack)
// library-internal flag of spgemm_impl: stop after the symbolic pass and the scan (cbg_estimate): the result holds the
// colptr only, nnz(C) and the multiplies are exact, no output is allocated or computed
constexpr uint32_t kSymbolicOnly = 1u << 28;

// Grow-only buffers.  `gen` counts reallocations: a pointer taken with as<T>() is stale once gen moves (the old block
// is freed, or handed back to the pool while kernels queued on the stream may still use it).  Captures records the
// generations of the buffers a phase's launches were given and check() refuses to launch after any of them moved.
struct DevBuf {
  void* p = nullptr;
  size_t n = 0;
  uint32_t gen = 0;
  ~DevBuf() { if (p) (void)hipFree(p); }
  hipError_t reserve(size_t bytes) {
    if (bytes <= n) return hipSuccess;
    ++gen;
    if (p) { (void)hipFree(p); p = nullptr; n = 0; }
    hipError_t e = hipMalloc(&p, bytes ? bytes : 16);
    if (e == hipSuccess) n = bytes;
    return e;
  }
  template <typename T> T* as() const { return (T*)p; }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    ++gen;
  }
};

inline size_t dt_size(cbg_dtype t) {
  switch (t) { case CBG_BOOL: return 1; case CBG_I32: case CBG_F32: return 4; default: return 8; }
}

template <typename V> struct DtOf;
template <> struct DtOf<double> { static constexpr cbg_dtype value = CBG_F64; };
template <> struct DtOf<float> { static constexpr cbg_dtype value = CBG_F32; };
template <> struct DtOf<int64_t> { static constexpr cbg_dtype value = CBG_I64; };
template <> struct DtOf<int32_t> { static constexpr cbg_dtype value = CBG_I32; };
template <> struct DtOf<uint8_t> { static constexpr cbg_dtype value = CBG_BOOL; };

// Caching pool for result storage.  A product's output is gigabytes at scale 20 and a fresh
// hipMalloc/hipFree of it costs far more than the product; like PyTorch's caching allocator, freed
// result blocks are kept per context and handed to the next result that fits (within 1.5x).
struct Pool {
  std::multimap<size_t, void*> free_;
  ~Pool() { trim(); }
  hipError_t get(size_t bytes, void** p, size_t* cap) {
    auto it = free_.lower_bound(bytes);
    if (it != free_.end() && it->first <= bytes + bytes / 2 + (1u << 20)) {
      *p = it->second;
      *cap = it->first;
      free_.erase(it);
      return hipSuccess;
    }
    hipError_t e = hipMalloc(p, bytes);
    if (e != hipSuccess && !free_.empty()) {   // give cached blocks back and retry once
      (void)hipGetLastError();
      trim();
      e = hipMalloc(p, bytes);
    }
    if (e == hipSuccess) *cap = bytes;
    return e;
  }
  void put(void* p, size_t cap) { free_.emplace(cap, p); }
  void trim() {
    for (auto& kv : free_) (void)hipFree(kv.second);
    free_.clear();
  }
};

struct PoolBuf {
  std::shared_ptr<Pool> pool;
  void* p = nullptr;
  size_t n = 0;
  uint32_t gen = 0;
  ~PoolBuf() { if (p) pool->put(p, n); }
  hipError_t reserve(size_t bytes) {
    if (bytes <= n) return hipSuccess;
    ++gen;
    if (p) { pool->put(p, n); p = nullptr; n = 0; }
    return pool->get(bytes ? bytes : 16, &p, &n);
  }
  template <typename T> T* as() const { return (T*)p; }
};

// Generations of the buffers whose pointers a phase captured; check() before the phase's launches.  A moved buffer
// is a host-side bug (a reserve after the capture): refuse the launch instead of handing kernels a freed block.
struct Captures {
  struct Ent { const uint32_t* gen; uint32_t at; const char* what; };
  std::vector<Ent> v;
  template <class Buf> void add(const Buf& b, const char* what) { v.push_back(Ent{&b.gen, b.gen, what}); }
  bool ok(const char** which = nullptr) const {
    for (const Ent& e : v)
      if (*e.gen != e.at) { if (which) *which = e.what; return false; }
    return true;
  }
};

// Synchronises the given streams when it goes out of scope.  Declared after the pool buffers that kernels or
// RCCL calls still in flight may touch, it runs before their destructors hand them back to the pool, on the
// error returns (HIPCHK / CBGCHK) as on the normal path.
struct StreamFence {
  hipStream_t a = nullptr, b = nullptr;
  StreamFence(hipStream_t x, hipStream_t y = nullptr) : a(x), b(y) {}
  ~StreamFence() {
    if (a) (void)hipStreamSynchronize(a);
    if (b) (void)hipStreamSynchronize(b);
  }
};

struct Owner {                 // device storage behind a cbg_csc_result
  PoolBuf cp, ir, val;
  explicit Owner(const std::shared_ptr<Pool>& pl) { cp.pool = ir.pool = val.pool = pl; }
};

}  // namespace host
}  // namespace cbg

using namespace cbg::host;

struct cbg_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  hipEvent_t ev[8] = {};
  std::shared_ptr<Pool> pool = std::make_shared<Pool>();
  cbg_profile prof{};
  // workspace (grow-only)
  DevBuf flop, span, cnt, list, hist, cursor, scan_tiles, scalars, cur, nxt, ovf_list, stageA[5], stageB[5];
  DevBuf split_idx, long_cols, split_tab, heavy_cols, sub, units, ucnt, uspan, ulist, fb_units, fb_list, uovf_list;
  DevBuf nunits, segsz, segoff, useg, icnt, itemoff, items, parts, wide_win;
  DevBuf hrows, hmode, hpoff, urows;   // symbolic -> numeric row handoff of heavy columns
  DevBuf oitems;                       // heavy items the rows-known kernel does not take
  DevBuf items2, ubkt;                 // the rows-known units in first-subwindow order + bucket counters (CBG_KNOWN_SORT)
  DevBuf ptab;                         // A's part table for k_sym_part (k_part_table)
  DevBuf acol;                         // A's (length, first row, last row) per column (k_acol_info)
  DevBuf aos;                          // A's rows and values interleaved (k_num_heavy_known gathers)
  DevBuf gal[9];                       // fused Galerkin product scratch (galerkin.hip)
  void* pin = nullptr;                 // 16 KB of pinned host memory: small read-backs (bin counts, scalars)
  int ncu = 0;                         // compute units (persistent grids)
  int lds_per_cu = 0;                  // LDS bytes per CU (hipDeviceAttributeMaxSharedMemoryPerMultiprocessor)
  int reserve_cu = 0;                  // CUs the persistent grids leave free (a concurrent RCCL transfer)
  int row_handoff = -1;                // -1: read CBG_ROW_HANDOFF once (default on)
};

// Give the grow-only product workspace (the symbolic row handoff alone is ~11 GB at s20) and the pool's cached
// blocks back to the device: called when an output that must fit next to large live pieces (the fiber merge at
// N = 2, s21) would not.  Synchronises the context's stream first.
inline void release_workspace(cbg_ctx* c) {
  (void)hipStreamSynchronize(c->stream);
  for (DevBuf* b : {&c->flop, &c->span, &c->cnt, &c->list, &c->hist, &c->cursor, &c->scan_tiles, &c->cur, &c->nxt,
                    &c->ovf_list, &c->split_idx, &c->long_cols, &c->split_tab, &c->heavy_cols, &c->sub, &c->units,
                    &c->ucnt, &c->uspan, &c->ulist, &c->fb_units, &c->fb_list, &c->uovf_list, &c->nunits, &c->segsz,
                    &c->segoff, &c->useg, &c->icnt, &c->itemoff, &c->items, &c->parts, &c->wide_win, &c->hrows,
                    &c->hmode, &c->hpoff, &c->urows, &c->oitems, &c->aos, &c->ptab, &c->items2, &c->ubkt, &c->acol})
    b->release();
  for (DevBuf& b : c->stageA) b.release();
  for (DevBuf& b : c->stageB) b.release();
  for (DevBuf& b : c->gal) b.release();
  c->pool->trim();
}

// pinned read-back slots (byte offsets into ctx->pin); a D2H copy into pageable memory goes through a staging
// buffer and costs tens of microseconds per host sync on small products
constexpr size_t kPinMerge = 2624, kPinMirror = 4096, kPinBytes = 16384;
template <typename T>
inline T* pinned(cbg_ctx* c, size_t off) { return (T*)((char*)c->pin + off); }

inline hipError_t launch_cfg_lds(const void* fn, size_t lds) {
  if (lds > 64 * 1024) return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  return hipSuccess;
}

// ------------------------------------------------------------------------------- input staging
namespace cbg { namespace host {
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

// ------------------------------------------------------------------------------- binning
struct Classes {
  std::vector<unsigned long long> hist;   // per class counts (+ [31] = items above the heavy bound)
  std::vector<unsigned long long> off;    // exclusive offsets
};

// pass 0 of a binning into hist_dev[0..63] (no sync); flop: lane-class test when cnt is not the flop
inline void bin_count(hipStream_t st, int64_t n, const int64_t* cnt, const int2* span, const int64_t* flop,
                      BinParams bp, unsigned long long* hist_dev, int32_t* list) {
  const int64_t g = (n + 256 * kBinPer - 1) / (256 * kBinPer);
  if (g > 0) k_bin<<<(int)g, 256, 0, st>>>(n, cnt, span, flop, bp, 0, kHeavy, hist_dev, hist_dev + 32, list);
}
// after the host has hist: offsets (the regular classes contiguous in class order, then the lane
// class) and pass 1, which derives the same offsets on the device (its cursors hist_dev[32..63] start at zero)
inline cbg_status bin_fill(hipStream_t st, int64_t n, const int64_t* cnt, const int2* span, const int64_t* flop,
                           BinParams bp, unsigned long long* hist_dev, const unsigned long long* hist_host,
                           int32_t* list, Classes* cl) {
  const int ncls = bp.nwave + bp.nblock + 2;
  cl->hist.assign(hist_host, hist_host + 32);
  cl->off.assign(32, 0);
  unsigned long long acc = 0;
  for (int c = 0; c < ncls; ++c) { cl->off[c] = acc; acc += cl->hist[c]; }
  cl->off[kLane8Class] = acc;
  acc += cl->hist[kLane8Class];
  cl->off[kLaneClass] = acc;
  const int64_t g = (n + 256 * kBinPer - 1) / (256 * kBinPer);
  if (g > 0) k_bin<<<(int)g, 256, 0, st>>>(n, cnt, span, flop, bp, 1, kHeavy, hist_dev, hist_dev + 32, list);
  return CBG_OK;
}

// ------------------------------------------------------------------------------- launch helpers
template <int LOGT>
void launch_sym_wave(hipStream_t st, const int32_t* l, int64_t n, const int64_t* Acp, const int32_t* Air,
                     const int64_t* Bcp, const int32_t* Bir, const int2* span, int64_t* nnz, const HeavyOut& ho) {
  k_sym_wave<LOGT><<<(int)grid_for(n, 4, kMaxGrid * 2), 256, 0, st>>>(l, n, Acp, Air, Bcp, Bir, span, nnz, ho);
}
template <int LOGT, int NT>
hipError_t launch_sym_block(hipStream_t st, const int32_t* l, int64_t n, const int64_t* Acp, const int32_t* Air,
                            const int64_t* Bcp, const int32_t* Bir, const int2* span, int64_t* nnz,
                            const HeavyOut& ho) {
  const size_t lds = sym_block_lds<LOGT, NT>();
  hipError_t e = launch_cfg_lds((const void*)k_sym_block<LOGT, NT>, lds);
  if (e != hipSuccess) return e;
  k_sym_block<LOGT, NT><<<(int)grid_for(n, 1, kMaxGrid), NT, lds, st>>>(l, n, Acp, Air, Bcp, Bir, span, nnz, ho);
  return hipGetLastError();
}
template <int NT>
hipError_t launch_sym_part(hipStream_t st, const PartItem* items, const int* count_dev, int64_t cap, int64_t annz,
                           const int64_t* Acp, const int32_t* Air, const int64_t* Bcp, const int32_t* Bir,
                           const int2* span, const Split& spl, int64_t* nnz, const HeavyOut& ho) {
  // 16-byte row loads (RowLd4) unless CBG_SYM_VEC4=0 or A has fewer than 4 entries; 32-bit segment staging (8 waves
  // per SIMD) unless A.nnz >= 2^31
  static const bool vec_env = [] { const char* e = std::getenv("CBG_SYM_VEC4"); return !(e && e[0] == '0'); }();
  const bool vec = vec_env && kGroupSym == 4 && annz >= 4;
  const bool w32 = annz < INT32_MAX;
  const size_t lds = w32 ? sym_part_lds<NT, int32_t>() : sym_part_lds<NT, int64_t>();
  const void* kf = w32 ? (vec ? (const void*)k_sym_part<NT, true, int32_t> : (const void*)k_sym_part<NT, false, int32_t>)
                       : (vec ? (const void*)k_sym_part<NT, true, int64_t> : (const void*)k_sym_part<NT, false, int64_t>);
  hipError_t e = launch_cfg_lds(kf, lds);
  if (e != hipSuccess) return e;
  const int g = (int)grid_for(cap, 1, kSymPartGrid);
  if (w32 && vec)
    k_sym_part<NT, true, int32_t><<<g, NT, lds, st>>>(items, count_dev, annz, Acp, Air, Bcp, Bir, span, spl, nnz, ho);
  else if (w32)
    k_sym_part<NT, false, int32_t><<<g, NT, lds, st>>>(items, count_dev, annz, Acp, Air, Bcp, Bir, span, spl, nnz, ho);
  else if (vec)
    k_sym_part<NT, true, int64_t><<<g, NT, lds, st>>>(items, count_dev, annz, Acp, Air, Bcp, Bir, span, spl, nnz, ho);
  else
    k_sym_part<NT, false, int64_t><<<g, NT, lds, st>>>(items, count_dev, annz, Acp, Air, Bcp, Bir, span, spl, nnz, ho);
  return hipGetLastError();
}
template <int LOGT, class SRT, typename V, bool UNIT>
void launch_num_wave(hipStream_t st, const int32_t* l, int64_t n, const Unit* units, const DevCsc<V>& A,
                     const DevCsc<V>& B, const int2* span, const int64_t* colptr, const Split& spl,
                     const NumOut<V>& o) {
  k_num_wave<SRT, V, LOGT, UNIT><<<(int)grid_for(n, 4, kMaxGrid * 2), 256, 0, st>>>(l, n, units, A, B, span, colptr,
                                                                                    spl, o);
}
template <int LOGT, int NT, class SRT, typename V, bool UNIT>
hipError_t launch_num_block(hipStream_t st, const int32_t* l, const int* n_dev, int64_t n, int64_t grid,
                            const Unit* units, const DevCsc<V>& A, const DevCsc<V>& B, const int2* span,
                            const int64_t* colptr, const Split& spl, const NumOut<V>& o) {
  const size_t lds = num_block_lds<SRT, V, LOGT, NT>();
  hipError_t e = launch_cfg_lds((const void*)k_num_block<SRT, V, LOGT, NT, UNIT>, lds);
  if (e != hipSuccess) return e;
  k_num_block<SRT, V, LOGT, NT, UNIT><<<(int)grid, NT, lds, st>>>(l, n_dev, n, units, A, B, span, colptr, spl, o);
  return hipGetLastError();
}
// persistent launches over device-counted lists: `grid` workgroups (one per CU; the LDS allows one)
template <int LOGT, int NT, class SRT, typename V>
hipError_t launch_num_heavy(hipStream_t st, int grid, const HeavyItem* items, const unsigned long long* nitems,
                            const int32_t* hcols, const Unit* units, int32_t nsub, const DevCsc<V>& A,
                            const DevCsc<V>& B, const int2* span, const Split& spl, const NumOut<V>& o,
                            unsigned long long* ticket) {
  if (grid <= 0) return hipSuccess;
  const size_t lds = num_heavy_lds<SRT, V, LOGT, NT>();
  hipError_t e = launch_cfg_lds((const void*)k_num_heavy<SRT, V, LOGT, NT>, lds);
  if (e != hipSuccess) return e;
  k_num_heavy<SRT, V, LOGT, NT><<<grid, NT, lds, st>>>(items, nitems, hcols, units, nsub, A, B, span, spl, o, ticket);
  return hipGetLastError();
}
template <int LOGT, int NT, class SRT, typename V>
hipError_t launch_num_heavy_known(hipStream_t st, int grid, const KnownUnit* ku, const unsigned long long* nku,
                                  const DevCsc<V>& A, const DevCsc<V>& B, const Split& spl, const NumOut<V>& o,
                                  unsigned long long* ticket, const RowVal<V>* arv = nullptr) {
  if (grid <= 0) return hipSuccess;
  const size_t lds = num_heavy_known_lds<SRT, V, LOGT, NT>();
  if (A.val && arv) {
    hipError_t e = launch_cfg_lds((const void*)k_num_heavy_known<SRT, V, LOGT, NT, true, true>, lds);
    if (e != hipSuccess) return e;
    k_num_heavy_known<SRT, V, LOGT, NT, true, true><<<grid, NT, lds, st>>>(ku, nku, A, B, spl, o, ticket, arv);
  } else if (A.val) {
    hipError_t e = launch_cfg_lds((const void*)k_num_heavy_known<SRT, V, LOGT, NT, true>, lds);
    if (e != hipSuccess) return e;
    k_num_heavy_known<SRT, V, LOGT, NT, true><<<grid, NT, lds, st>>>(ku, nku, A, B, spl, o, ticket);
  } else {
    hipError_t e = launch_cfg_lds((const void*)k_num_heavy_known<SRT, V, LOGT, NT, false>, lds);
    if (e != hipSuccess) return e;
    k_num_heavy_known<SRT, V, LOGT, NT, false><<<grid, NT, lds, st>>>(ku, nku, A, B, spl, o, ticket);
  }
  return hipGetLastError();
}
template <int MODE, class SRT, typename V, int W>
hipError_t launch_window(hipStream_t st, const int32_t* l, const int* count_dev, int64_t count_host, int64_t grid,
                         const DevCsc<V>& A, const DevCsc<V>& B, const int2* span, const int64_t* colptr,
                         int64_t* cur, int32_t* nxt, int64_t* nnz, const HeavyOut& ho, const NumOut<V>& o) {
  const size_t lds = window_lds<MODE, SRT, V, kWinNT, W>();
  hipError_t e = launch_cfg_lds((const void*)k_window<MODE, SRT, V, kWinNT, W>, lds);
  if (e != hipSuccess) return e;
  k_window<MODE, SRT, V, kWinNT, W><<<(int)grid, kWinNT, lds, st>>>(l, count_dev, count_host, A, B, span, colptr, cur,
                                                                    nxt, nnz, ho, o);
  return hipGetLastError();
}

// numeric kernels over one binned list (columns, or units when UNIT)
template <class SRT, typename V, bool UNIT>
hipError_t launch_numeric_classes(hipStream_t st, const Classes& cl, const int32_t* list, const Unit* units,
                                  const DevCsc<V>& A, const DevCsc<V>& B, const int2* span, const int64_t* colptr,
                                  const Split& spl, const NumOut<V>& o) {
  auto L = [&](int c) { return list + cl.off[c]; };
  auto n = [&](int c) { return (int64_t)cl.hist[c]; };
  if constexpr (!UNIT) {
    if (n(kLane8Class))
      k_num_lane<SRT, V, kLaneSmall><<<(int)grid_for(n(kLane8Class), 256, kMaxGrid * 4), 256, 0, st>>>(
          L(kLane8Class), n(kLane8Class), A, B, colptr, o);
    if (n(kLaneClass))
      k_num_lane<SRT, V, kLaneMax><<<(int)grid_for(n(kLaneClass), 256, kMaxGrid * 4), 256, 0, st>>>(L(kLaneClass), n(kLaneClass),
                                                                                          A, B, colptr, o);
  }
  if (n(1)) launch_num_wave<6, SRT, V, UNIT>(st, L(1), n(1), units, A, B, span, colptr, spl, o);
  if (n(2)) launch_num_wave<7, SRT, V, UNIT>(st, L(2), n(2), units, A, B, span, colptr, spl, o);
  if (n(3)) launch_num_wave<8, SRT, V, UNIT>(st, L(3), n(3), units, A, B, span, colptr, spl, o);
  if (n(4)) launch_num_wave<9, SRT, V, UNIT>(st, L(4), n(4), units, A, B, span, colptr, spl, o);
  hipError_t e = hipSuccess;
  if (n(5) && e == hipSuccess)
    e = launch_num_block<10, 256, SRT, V, UNIT>(st, L(5), nullptr, n(5), grid_for(n(5), 1, kMaxGrid), units, A, B,
                                                span, colptr, spl, o);
  if (n(6) && e == hipSuccess)
    e = launch_num_block<11, 256, SRT, V, UNIT>(st, L(6), nullptr, n(6), grid_for(n(6), 1, kMaxGrid), units, A, B,
                                                span, colptr, spl, o);
  if (n(7) && e == hipSuccess)
    e = launch_num_block<12, 512, SRT, V, UNIT>(st, L(7), nullptr, n(7), grid_for(n(7), 1, kMaxGrid), units, A, B,
                                                span, colptr, spl, o);
  if (n(8) && e == hipSuccess)
    e = launch_num_block<13, 1024, SRT, V, UNIT>(st, L(8), nullptr, n(8), grid_for(n(8), 1, kMaxGrid), units, A, B,
                                                 span, colptr, spl, o);
  return e;
}

// ------------------------------------------------------------------------------- the product
template <class SRT, typename V>
cbg_status spgemm_impl(cbg_ctx* ctx, const cbg_dcsc_view* Av, const cbg_dcsc_view* Bv, uint32_t flags,
                       cbg_csc_result* C, int64_t* mult_out) {
  // output columns are always row-sorted (sorting is free in the compaction); kSymbolicOnly: cbg_estimate
  const bool symbolic_only = (flags & kSymbolicOnly) != 0;
  hipStream_t st = ctx->stream;
  cbg_profile& pf = ctx->prof;
  memset(&pf, 0, sizeof(pf));
  if (Av->ncol != Bv->nrow) return CBG_EDIM;
  const int64_t M = Av->nrow, N = Bv->ncol;
  // Select2nd / BoolCopy2nd accumulate the (int32) position of the contributing B nonzero
  if (SRT::kNeedsBPos && Bv->nnz >= (int64_t)INT32_MAX) return CBG_EUNSUP;

  std::unique_ptr<Owner> own(new Owner(ctx->pool));
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

  // subwindow geometry of the row space (heavy-column units)
  // SUBW >= 2^13: k_sym_part's per-part subwindow counters assume it, and a single-subwindow unit
  // must fit k_num_heavy's dense table (2^CBG_HEAVY_LOGT rows)
  static_assert(CBG_HEAVY_LOGT >= 12, "k_num_heavy table of at least 2^12 rows");
  int32_t slog = kSubLogMin;
  while (((M - 1) >> slog) + 1 > kMaxSub) ++slog;
  const int32_t nsub = (int32_t)(((M - 1) >> slog) + 1);

  // 1. column statistics
  HIPCHK(ctx->flop.reserve(sizeof(int64_t) * (N + 1)));
  HIPCHK(ctx->span.reserve(sizeof(int2) * (N + 1)));
  HIPCHK(ctx->cnt.reserve(sizeof(int64_t) * (N + 1)));
  HIPCHK(ctx->list.reserve(sizeof(int32_t) * (N + 1)));
  HIPCHK(ctx->hist.reserve(sizeof(unsigned long long) * 256));
  HIPCHK(ctx->scalars.reserve(256));
  HIPCHK(ctx->ovf_list.reserve(sizeof(int32_t) * (N + 1)));
  HIPCHK(ctx->split_idx.reserve(sizeof(int32_t) * (A.ncol + 1)));
  HIPCHK(ctx->long_cols.reserve(sizeof(int32_t) * (A.ncol + 1)));
  HIPCHK(ctx->acol.reserve(sizeof(int4) * (A.ncol + 1)));
  Captures cap;   // every workspace pointer below is taken after its buffer's last reserve; CAPCHK before launches
  cap.add(ctx->flop, "flop"); cap.add(ctx->span, "span"); cap.add(ctx->cnt, "cnt"); cap.add(ctx->list, "list");
  cap.add(ctx->hist, "hist"); cap.add(ctx->scalars, "scalars"); cap.add(ctx->ovf_list, "ovf_list");
  cap.add(ctx->split_idx, "split_idx"); cap.add(ctx->long_cols, "long_cols"); cap.add(ctx->acol, "acol");
  int64_t* flop = ctx->flop.as<int64_t>();
  int2* span = ctx->span.as<int2>();
  int64_t* nnz = ctx->cnt.as<int64_t>();
  int32_t* list = ctx->list.as<int32_t>();
  unsigned long long* hist = ctx->hist.as<unsigned long long>();
  // scalars: [0] multiplies, [1] nnz(C); ints from byte 16: heavy n, nlong, adderr, col ovf, unit ovf,
  // fallback units, fallback-unit ovf; [16..18] heavy multiplies, B nonzeros, outputs (k_heavy_sums)
  // the scalars sit right after the binning histogram and its cursors (hist[0..63]), so that one device-to-host
  // copy of hist[0..64+k) brings back both; pm mirrors that range in pinned host memory (pm[i] = hist[i])
  unsigned long long* sc = hist + 64;
  unsigned long long* pm = pinned<unsigned long long>(ctx, kPinMirror);
  const unsigned long long* psc = pm + 64;
  auto mirror = [&](int lo, int hi) {   // hist[lo..hi) -> pm[lo..hi)
    return hipMemcpyAsync(pm + lo, hist + lo, sizeof(unsigned long long) * (hi - lo), hipMemcpyDeviceToHost, st);
  };
  int* si = (int*)(sc + 2);
  int *heavy_n = si + 0, *nlong = si + 1, *adderr = si + 2, *ovf_n = si + 3, *uovf_n = si + 4, *fb_n = si + 5,
      *fb_ovf_n = si + 6;
  HIPCHK(hipMemsetAsync(hist, 0, sizeof(unsigned long long) * 96, st));   // the symbolic histogram and sc together
  HIPCHK(hipMemsetAsync(nnz, 0, sizeof(int64_t) * N, st));
  {
    int4* ainfo = ctx->acol.as<int4>();
    k_acol_info<<<(int)std::max<int64_t>(1, std::min<int64_t>(kMaxGrid, (A.ncol + 1023) / 1024)), 256, 0, st>>>(
        A.ncol, A.cp, A.ir, ainfo, ctx->split_idx.as<int32_t>(), ctx->long_cols.as<int32_t>(), nlong);
    const int64_t avg = N > 0 ? (B.nnz + N - 1) / N : 0;   // lanes per column ~ the mean B column length
    if (avg <= 4)
      k_col_stats<4><<<(int)grid_for(N * 4, 256, kMaxGrid), 256, 0, st>>>(N, ainfo, B.cp, B.ir, flop, span, sc);
    else if (avg <= 8)
      k_col_stats<8><<<(int)grid_for(N * 8, 256, kMaxGrid), 256, 0, st>>>(N, ainfo, B.cp, B.ir, flop, span, sc);
    else
      k_col_stats<16><<<(int)grid_for(N * 16, 256, kMaxGrid), 256, 0, st>>>(N, ainfo, B.cp, B.ir, flop, span, sc);
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(ctx->ev[1], st));

  // 2. symbolic binning + kernels
  Classes cs;
  BinParams sbp{kSymWave, kSymBlock, 64, 1, kLaneMax};
  bin_count(st, N, flop, span, nullptr, sbp, hist, list);   // (hist zeroed with sc above)
  HIPCHK(mirror(0, 64 + 12));   // the class counts and sc[0..11]
  HIPCHK(hipStreamSynchronize(st));
  const int NL = ((const int*)&psc[2])[1];
  if ((s = bin_fill(st, N, flop, span, nullptr, sbp, hist, pm, list, &cs)) != CBG_OK) return s;
  const int64_t hcap = (int64_t)cs.hist[31];
  HIPCHK(ctx->heavy_cols.reserve(sizeof(int32_t) * (hcap + 1)));
  HIPCHK(ctx->sub.reserve(sizeof(int32_t) * (hcap * nsub + 1)));
  cap.add(ctx->heavy_cols, "heavy_cols"); cap.add(ctx->sub, "sub");
  HeavyOut ho{heavy_n, ctx->heavy_cols.as<int32_t>(), ctx->sub.as<int32_t>(), nsub, slog,
              nullptr, nullptr, 0, nullptr, nullptr, 0};
  // row handoff: scratch for the heavy columns' sorted rows, sized by the bound sum(min(flop, span))
  // over flop-heavy columns (k_col_stats); off if that does not fit comfortably in free memory
  if (ctx->row_handoff < 0) {
    const char* e = getenv("CBG_ROW_HANDOFF");
    ctx->row_handoff = (e && e[0] == '0') ? 0 : 1;
  }
  const unsigned long long hbound = psc[10];
  if (ctx->row_handoff && hcap > 0 && hbound > 0 && !SRT::kAddIsError && !symbolic_only) {
    size_t fr = 0, tot = 0;
    HIPCHK(hipMemGetInfo(&fr, &tot));
    // k_sym_part reserves rows per workgroup in chunks: it drops at most 1/7 of the rows it places (a leftover < chunk/8
    // per chunk at least 7/8 used) plus one chunk per workgroup (at most kSymPartGrid); + a pad
    int64_t chunk = std::min<int64_t>(16384, (int64_t)hbound / (4 * kSymPartGrid));
    if (chunk < 512) chunk = 0;
    const unsigned long long hcapr = hbound + (chunk ? hbound / 7 + 1 : 0) + (unsigned long long)(kSymPartGrid * chunk);
    const size_t need = sizeof(HRow) * (hcapr + 2);
    if (need <= ctx->hrows.n || need < fr / 3) {
      HIPCHK(ctx->hrows.reserve(need));
      HIPCHK(ctx->hmode.reserve(sizeof(int32_t) * (hcap + 1)));
      HIPCHK(ctx->hpoff.reserve(sizeof(int64_t) * (hcap * kMaxParts + 1)));
      HIPCHK(hipMemsetAsync(ctx->hmode.p, 0, sizeof(int32_t) * (hcap + 1), st));
      ho.rows = ctx->hrows.as<HRow>();
      ho.cursor = sc + 11;
      ho.cap = hcapr;
      ho.chunk = chunk;
      ho.poff = ctx->hpoff.as<int64_t>();
      ho.mode = ctx->hmode.as<int32_t>();
      cap.add(ctx->hrows, "hrows"); cap.add(ctx->hmode, "hmode"); cap.add(ctx->hpoff, "hpoff");
    }
  }
  // split table (unit segments, wide-column parts): needed whenever a column can be heavy
  Split spl{ctx->split_idx.as<int32_t>(), nullptr, nsub, slog, nullptr, nullptr, nullptr, nullptr, 0};
  if (hcap > 0) {
    HIPCHK(ctx->split_tab.reserve(sizeof(int32_t) * ((int64_t)NL * (nsub + 1) + 1)));
    spl.tab = ctx->split_tab.as<int32_t>();
    cap.add(ctx->split_tab, "split_tab");
    if (NL > 0)
      k_split_fill<<<(int)grid_for(NL, 4, kMaxGrid * 2), 256, 0, st>>>(NL, ctx->long_cols.as<int32_t>(), A.cp, A.ir,
                                                                        ctx->split_tab.as<int32_t>(), nsub, slog);
  }
  HIPCHK(hipEventRecord(ctx->ev[2], st));
  CAPCHK(cap);
  {
    auto L = [&](int c) { return list + cs.off[c]; };
    auto n = [&](int c) { return (int64_t)cs.hist[c]; };
    if (n(kLaneClass))
      k_sym_lane<<<(int)grid_for(n(kLaneClass), 256, kMaxGrid * 4), 256, 0, st>>>(L(kLaneClass), n(kLaneClass), A.cp,
                                                                                  A.ir, B.cp, B.ir, nnz);
    if (n(1)) launch_sym_wave<6>(st, L(1), n(1), A.cp, A.ir, B.cp, B.ir, span, nnz, ho);
    if (n(2)) launch_sym_wave<7>(st, L(2), n(2), A.cp, A.ir, B.cp, B.ir, span, nnz, ho);
    if (n(3)) launch_sym_wave<8>(st, L(3), n(3), A.cp, A.ir, B.cp, B.ir, span, nnz, ho);
    if (n(4)) launch_sym_wave<9>(st, L(4), n(4), A.cp, A.ir, B.cp, B.ir, span, nnz, ho);
    if (n(5)) launch_sym_wave<10>(st, L(5), n(5), A.cp, A.ir, B.cp, B.ir, span, nnz, ho);
    hipError_t e = hipSuccess;
    if (n(6) && e == hipSuccess) e = launch_sym_block<11, 256>(st, L(6), n(6), A.cp, A.ir, B.cp, B.ir, span, nnz, ho);
    if (n(7) && e == hipSuccess) e = launch_sym_block<12, 256>(st, L(7), n(7), A.cp, A.ir, B.cp, B.ir, span, nnz, ho);
    if (n(8) && e == hipSuccess) e = launch_sym_block<13, 512>(st, L(8), n(8), A.cp, A.ir, B.cp, B.ir, span, nnz, ho);
    // wide columns (classes kWideClass..11, contiguous in the list): (column, part) items; the
    // widest (more than kMaxParts parts), or all of them when a subwindow is larger than a part
    // (nrow > 2^(kPartLog+11)), go to the windowed kernel
    if (kWideClass > 9 && n(9) && e == hipSuccess)
      e = launch_sym_block<14, 1024>(st, L(9), n(9), A.cp, A.ir, B.cp, B.ir, span, nnz, ho);
    int64_t nwide = 0;
    for (int c = kWideClass; c <= 11; ++c) nwide += n(c);
    if (nwide && e == hipSuccess) {
      HIPCHK(ctx->parts.reserve(sizeof(PartItem) * (nwide * kMaxParts + 1)));
      HIPCHK(ctx->wide_win.reserve(sizeof(int32_t) * (nwide + 1)));
      cap.add(ctx->parts, "parts"); cap.add(ctx->wide_win, "wide_win");
      // the part table of A (k_part_table), unless it would not fit comfortably (CBG_PART_TABLE=0: off)
      static const bool ptab_env = [] { const char* x = std::getenv("CBG_PART_TABLE"); return !(x && x[0] == '0'); }();
      const int32_t P = (int32_t)(((M - 1) >> kPartLog) + 1);
      int32_t PS = 8;   // row stride in words: a power of two >= P + 3 (k_part_table)
      while (PS < P + 3) PS <<= 1;
      const size_t pbytes = sizeof(int32_t) * ((size_t)A.ncol * PS + 1);
      size_t pfree = 0, ptot = 0;
      if (ptab_env && P > 1 && A.ncol > 0 &&
          (pbytes <= ctx->ptab.n || (hipMemGetInfo(&pfree, &ptot) == hipSuccess && pbytes < pfree / 8))) {
        HIPCHK(ctx->ptab.reserve(pbytes));
        cap.add(ctx->ptab, "ptab");
        k_part_table<<<(int)grid_for(A.ncol, 256, kMaxGrid * 4), 256, 0, st>>>(A.ncol, A.cp, A.ir, P, PS,
                                                                                 ctx->ptab.as<int32_t>());
        spl.ptab = ctx->ptab.as<int32_t>();
        spl.pstride = PS;
      }
      CAPCHK(cap);
      int *nparts = si + 8, *nwin = si + 9;
      k_part_items<<<(int)grid_for(nwide, 256, kMaxGrid), 256, 0, st>>>(L(kWideClass), nwide, slog <= kPartLog ? kMaxParts : 0, span, ho,
                                                                         ctx->parts.as<PartItem>(), nparts,
                                                                         ctx->wide_win.as<int32_t>(), nwin);
      e = launch_sym_part<kPartNT>(st, ctx->parts.as<PartItem>(), nparts, nwide * kMaxParts, A.nnz, A.cp, A.ir, B.cp, B.ir,
                               span, spl, nnz, ho);
      const int64_t nw_cap = slog <= kPartLog ? n(11) : nwide;
      if (nw_cap && e == hipSuccess) {
        HIPCHK(ctx->cur.reserve(sizeof(int64_t) * (B.nnz + 1)));
        HIPCHK(ctx->nxt.reserve(sizeof(int32_t) * (B.nnz + 1)));
        CAPCHK(cap);
        e = launch_window<0, SRT, V, kSymWinRows>(st, ctx->wide_win.as<int32_t>(), nwin, nw_cap,
                                                  grid_for(nw_cap, 1, 1024), A, B, span, nullptr,
                                                  ctx->cur.as<int64_t>(), ctx->nxt.as<int32_t>(), nnz, ho,
                                                  NumOut<V>{});
      }
    }
    if (e != hipSuccess) { fprintf(stderr, "cbgpu: symbolic launch: %s\n", hipGetErrorString(e)); return CBG_EDEVICE; }
    HIPCHK(hipGetLastError());
  }
  HIPCHK(hipEventRecord(ctx->ev[3], st));

  // 3. scan -> colptr, nnz(C)
  const int64_t ntiles = (N + kScanTile - 1) / kScanTile;
  HIPCHK(ctx->scan_tiles.reserve(sizeof(int64_t) * (ntiles + 1)));
  cap.add(ctx->scan_tiles, "scan_tiles");
  CAPCHK(cap);
  k_scan_tiles<<<(int)ntiles, 256, 0, st>>>(N, nnz, ctx->scan_tiles.as<int64_t>());
  k_scan_sums<<<1, 1024, 0, st>>>(ntiles, ctx->scan_tiles.as<int64_t>(), (int64_t*)(sc + 1));
  k_scan_apply<<<(int)ntiles, 256, 0, st>>>(N, nnz, ctx->scan_tiles.as<int64_t>(), colptr);
  HIPCHK(hipGetLastError());
  // no column can be heavy (hcap = 0 columns above kHeavy multiplies): the numeric binning needs nothing from
  // the host, so its histogram comes back with nnz(C) in the same read-back (three host syncs per product)
  const bool early_nbin = !symbolic_only && hcap == 0;
  BinParams nbp{kNumWave, kNumBlock, 64, 0, kLaneMax};
  auto numeric_bin_count = [&]() -> hipError_t {   // (hist[0..63] only: sc follows)
    hipError_t e = hipMemsetAsync(hist, 0, sizeof(unsigned long long) * 64, st);
    if (e == hipSuccess) bin_count(st, N, nnz, span, flop, nbp, hist, list);
    return e;
  };
  if (early_nbin) {
    HIPCHK(numeric_bin_count());
    HIPCHK(mirror(0, 64 + 4));   // the numeric class counts and sc[0..3]
  } else {
    HIPCHK(mirror(64, 64 + 4));
  }
  HIPCHK(hipStreamSynchronize(st));
  const unsigned long long* hsc = psc;
  HIPCHK(hipEventRecord(ctx->ev[4], st));
  const int64_t mults = (int64_t)hsc[0], nnzc = (int64_t)hsc[1];
  const int H = ((int*)&hsc[2])[0];
  if (early_nbin && H > 0) {   // a heavy column has nnz <= flop above kHeavy, so hcap = 0 rules it out
    fprintf(stderr, "cbgpu: %d heavy columns with no column above the heavy bound\n", H);
    return CBG_EDEVICE;
  }
  pf.multiplies = mults; pf.nnz_out = nnzc;
  if (symbolic_only) {
    HIPCHK(own->ir.reserve(4));
    HIPCHK(own->val.reserve(8));
    float t;
    (void)hipEventElapsedTime(&t, ctx->ev[0], ctx->ev[1]); pf.flops_ms = t;
    (void)hipEventElapsedTime(&t, ctx->ev[1], ctx->ev[2]); pf.bin_ms = t;
    (void)hipEventElapsedTime(&t, ctx->ev[2], ctx->ev[3]); pf.symbolic_ms = t;
    (void)hipEventElapsedTime(&t, ctx->ev[3], ctx->ev[4]); pf.scan_ms = t;
    (void)hipEventElapsedTime(&t, ctx->ev[0], ctx->ev[4]); pf.total_ms = t;
    C->nnz = nnzc;
    C->colptr = colptr;
    C->row = own->ir.as<int32_t>();
    C->val = own->val.p;
    C->multiplies = mults;
    C->_owner = own.release();
    if (mult_out) *mult_out = mults;
    return CBG_OK;
  }
  // what the heavy kernels will process (listed columns with nnz > kHeavy): sc[16..18], read back with the errors
  if (H > 0)
    k_heavy_sums<<<(int)grid_for(H, 256, 1024), 256, 0, st>>>(H, ctx->heavy_cols.as<int32_t>(), flop, nnz, B.cp, sc + 16);
  HIPCHK(own->ir.reserve(sizeof(int32_t) * (nnzc + 1)));
  HIPCHK(own->val.reserve(sizeof(V) * (nnzc + 1)));

  // 4. heavy columns -> units (split table + greedy subwindow grouping)
  const int64_t nunit_cap = (int64_t)H * nsub;
  Unit* units = nullptr;
  const KnownUnit* known_list = nullptr;   // the rows-known unit list the heavy kernel takes (items, or items2 sorted)
  if (H > 0) {
    HIPCHK(ctx->units.reserve(sizeof(Unit) * (nunit_cap + 1)));
    HIPCHK(ctx->ucnt.reserve(sizeof(int64_t) * (nunit_cap + 1)));
    HIPCHK(ctx->uspan.reserve(sizeof(int2) * (nunit_cap + 1)));
    HIPCHK(ctx->ulist.reserve(sizeof(int32_t) * (nunit_cap + 1)));
    HIPCHK(ctx->fb_units.reserve(sizeof(Unit) * (nunit_cap + 1)));
    HIPCHK(ctx->fb_list.reserve(sizeof(int32_t) * (nunit_cap + 1)));
    HIPCHK(ctx->uovf_list.reserve(sizeof(int32_t) * (nunit_cap + 1)));
    HIPCHK(hipMemsetAsync(ctx->ucnt.p, 0, sizeof(int64_t) * nunit_cap, st));
    units = ctx->units.as<Unit>();
    HIPCHK(ctx->nunits.reserve(sizeof(int32_t) * (H + 1)));
    HIPCHK(ctx->segsz.reserve(sizeof(int64_t) * (H + 1)));
    HIPCHK(ctx->segoff.reserve(sizeof(int64_t) * (H + 1)));
    HIPCHK(ctx->icnt.reserve(sizeof(int64_t) * (H + 1)));
    HIPCHK(ctx->itemoff.reserve(sizeof(int64_t) * (H + 1)));
    if (ho.rows) HIPCHK(ctx->urows.reserve(sizeof(UnitRows) * (nunit_cap + 1)));
    for (DevBuf* b : {&ctx->units, &ctx->ucnt, &ctx->uspan, &ctx->ulist, &ctx->fb_units, &ctx->fb_list, &ctx->uovf_list,
                      &ctx->nunits, &ctx->segsz, &ctx->segoff, &ctx->icnt, &ctx->itemoff, &ctx->urows})
      cap.add(*b, "heavy units");
    CAPCHK(cap);
    k_build_units<<<(H + 255) / 256, 256, 0, st>>>(H, ctx->heavy_cols.as<int32_t>(), ctx->sub.as<int32_t>(), nsub,
                                                   slog, heavy_unit_cap<SRT>(), heavy_span_cap<SRT>(),
                                                   heavy_rank_bytes<SRT>(), (int32_t)sizeof(typename SRT::Acc), span,
                                                   colptr, B.cp, units, ctx->ucnt.as<int64_t>(),
                                                   ctx->uspan.as<int2>(), nnz, ctx->nunits.as<int32_t>(),
                                                   ctx->segsz.as<int64_t>(), ctx->icnt.as<int64_t>(),
                                                   ho.mode, ho.poff,
                                                   ho.rows ? ctx->urows.as<UnitRows>() : nullptr);
    spl.hrows = ho.rows;
    spl.urows = ho.rows ? ctx->urows.as<UnitRows>() : nullptr;
    // offsets of every heavy column's block of (unit, B nonzero) segments; total -> sc[8]
    const int64_t ht = (H + kScanTile - 1) / kScanTile;
    k_scan_tiles<<<(int)ht, 256, 0, st>>>(H, ctx->segsz.as<int64_t>(), ctx->scan_tiles.as<int64_t>());
    k_scan_sums<<<1, 1024, 0, st>>>(ht, ctx->scan_tiles.as<int64_t>(), (int64_t*)(sc + 8));
    k_scan_apply<<<(int)ht, 256, 0, st>>>(H, ctx->segsz.as<int64_t>(), ctx->scan_tiles.as<int64_t>(),
                                          ctx->segoff.as<int64_t>());
    // the same for the heavy items (groups of kItemUnits units); total -> sc[9]
    k_scan_tiles<<<(int)ht, 256, 0, st>>>(H, ctx->icnt.as<int64_t>(), ctx->scan_tiles.as<int64_t>());
    k_scan_sums<<<1, 1024, 0, st>>>(ht, ctx->scan_tiles.as<int64_t>(), (int64_t*)(sc + 9));
    k_scan_apply<<<(int)ht, 256, 0, st>>>(H, ctx->icnt.as<int64_t>(), ctx->scan_tiles.as<int64_t>(),
                                          ctx->itemoff.as<int64_t>());
    HIPCHK(hipGetLastError());
  }

  // 5. numeric binning (columns and units, one host sync) + kernels; heavy items split into the
  //    rows-known list (k_num_heavy_known) and the rest (k_num_heavy), counts -> sc[12], sc[13]
  Classes cn;
  if (!early_nbin) {
    HIPCHK(numeric_bin_count());
    HIPCHK(mirror(0, 64 + 10));   // the numeric class counts and sc[8..9] (zero unless H > 0)
    HIPCHK(hipStreamSynchronize(st));
  }
  const unsigned long long* hn = pm;
  const int64_t segtot = (int64_t)psc[8], nitems = (int64_t)psc[9];
  if (H > 0) {
    HIPCHK(ctx->useg.reserve(sizeof(UnitSeg) * (segtot + 1)));
    spl.useg = ctx->useg.as<UnitSeg>();
    cap.add(ctx->useg, "useg");
    k_unit_segs<SRT, CBG_KNOWN_LOGT, CBG_KNOWN_NT><<<H, 256, 0, st>>>(
        ctx->heavy_cols.as<int32_t>(), ctx->nunits.as<int32_t>(), ctx->segoff.as<int64_t>(), units, nsub, A.cp,
        ctx->acol.as<int4>(), B.cp, B.ir, spl, ctx->useg.as<UnitSeg>());
    // units -> rows-known list + other items (device counts sc[12], sc[13]; units <= items * kItemUnits)
    const int64_t ucap = nitems * kItemUnits + 1;
    HIPCHK(ctx->items.reserve(sizeof(KnownUnit) * ucap));
    HIPCHK(ctx->oitems.reserve(sizeof(HeavyItem) * ucap));
    cap.add(ctx->items, "items"); cap.add(ctx->oitems, "oitems");
    CAPCHK(cap);
    k_heavy_items_split<SRT, CBG_KNOWN_LOGT, CBG_KNOWN_NT><<<(H + 255) / 256, 256, 0, st>>>(
        H, ctx->heavy_cols.as<int32_t>(), ctx->nunits.as<int32_t>(), units, nsub, slog, ctx->sub.as<int32_t>(),
        ctx->uspan.as<int2>(), spl.urows,
        B.cp, ctx->items.as<KnownUnit>(), ctx->oitems.as<HeavyItem>(), sc + 12);
    HIPCHK(hipGetLastError());
    known_list = ctx->items.as<KnownUnit>();
    // CBG_KNOWN_SORT=1: the rows-known units in first-subwindow order (k_known_bucket)
    static const bool ksort = [] { const char* x = std::getenv("CBG_KNOWN_SORT"); return x ? x[0] == '1' : CBG_KNOWN_SORT_DEFAULT != 0; }();
    if (ksort && nsub <= kMaxSub) {
      HIPCHK(ctx->items2.reserve(sizeof(KnownUnit) * ucap));
      HIPCHK(ctx->ubkt.reserve(sizeof(unsigned long long) * 3 * (nsub + 1)));
      cap.add(ctx->items2, "items2"); cap.add(ctx->ubkt, "ubkt");
      CAPCHK(cap);
      unsigned long long* bcnt = ctx->ubkt.as<unsigned long long>();
      unsigned long long* bbase = bcnt + (nsub + 1);
      unsigned long long* bcur = bbase + (nsub + 1);
      HIPCHK(hipMemsetAsync(bcnt, 0, sizeof(unsigned long long) * 3 * (nsub + 1), st));
      const int gs = (int)grid_for(ucap, kSortChunk, 4096);
      k_known_bucket<false><<<gs, kSortChunk, 0, st>>>(ctx->items.as<KnownUnit>(), sc + 12, slog, nsub, bcnt, nullptr,
                                                       nullptr, nullptr);
      k_known_bucket_base<<<1, 1024, 0, st>>>(nsub, bcnt, bbase);
      k_known_bucket<true><<<gs, kSortChunk, 0, st>>>(ctx->items.as<KnownUnit>(), sc + 12, slog, nsub, nullptr, bbase,
                                                      bcur, ctx->items2.as<KnownUnit>());
      HIPCHK(hipGetLastError());
      known_list = ctx->items2.as<KnownUnit>();
    }
  }
  if ((s = bin_fill(st, N, nnz, span, flop, nbp, hist, hn, list, &cn)) != CBG_OK) return s;
  if (cn.hist[kNumWave + kNumBlock + 1] != 0) {   // every column above kHeavy must have become units
    fprintf(stderr, "cbgpu: %llu unbinned numeric columns\n", (unsigned long long)cn.hist[kNumWave + kNumBlock + 1]);
    return CBG_EDEVICE;
  }
  for (int c = 0; c < 12; ++c) pf.bins[c] = (int64_t)cn.hist[c];
  pf.bins[12] = H;
  pf.bins[13] = nitems;
  NumOut<V> oc{own->ir.as<int32_t>(), own->val.as<V>(), adderr, ovf_n, ctx->ovf_list.as<int32_t>()};
  CAPCHK(cap);
  {
    hipError_t e = launch_numeric_classes<SRT, V, false>(st, cn, list, nullptr, A, B, span, colptr, spl, oc);
    if (e == hipSuccess && H > 0) {
      NumOut<V> ou{own->ir.as<int32_t>(), own->val.as<V>(), adderr, uovf_n, ctx->uovf_list.as<int32_t>()};
      HIPCHK(hipEventRecord(ctx->ev[6], st));
      if (ctx->ncu <= 0) {
        int ncu = 0, lds = 0;
        HIPCHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, ctx->device));
        HIPCHK(hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, ctx->device));
        ctx->ncu = ncu > 0 ? ncu : 256;
        ctx->lds_per_cu = lds > 0 ? lds : (160 << 10);
      }
      // persistent: as many workgroups as the LDS lets every CU hold (160 KB per CU on gfx950), less the CUs
      // reserved for a concurrent transfer (ctx->reserve_cu, set by the fiber pipeline while RCCL runs)
      const int per_cu =
          std::max<int>(1, (int)((size_t)ctx->lds_per_cu / num_heavy_known_lds<SRT, V, CBG_KNOWN_LOGT, CBG_KNOWN_NT>()));
      // CBG_HEAVY_RESERVE_CU: a standing reservation (tuning / tools/coresidency_probe.py)
      static const int reserve_env = [] { const char* x = std::getenv("CBG_HEAVY_RESERVE_CU"); return x ? atoi(x) : 0; }();
      const int cus = std::max(1, ctx->ncu - std::max(0, std::max(ctx->reserve_cu, reserve_env)));
      const int grid = (int)std::min<int64_t>((int64_t)cus * per_cu, nitems * kItemUnits);
      // CBG_AOS=1: A's rows and values interleaved for the rows-known kernel's gathers (one 16-byte load per
      // multiply).  Off by default: measured slower at s20 (heavy 34.3 vs 32.8 ms) and even at s21 (108.1 vs
      // 107.1 ms) -- the extra 4 bytes per gathered entry cost more than the halved load count saves
      const RowVal<V>* arv = nullptr;
      static const bool aos_env = [] { const char* x = std::getenv("CBG_AOS"); return x && x[0] == '1'; }();
      if (aos_env && A.val && sizeof(V) >= 4 && e == hipSuccess) {
        const size_t need = sizeof(RowVal<V>) * (size_t)(A.nnz + 1);
        size_t fr = 0, tot = 0;
        if (need <= ctx->aos.n || (hipMemGetInfo(&fr, &tot) == hipSuccess && need < fr / 4)) {
          HIPCHK(ctx->aos.reserve(need));
          k_pack_rowval<V><<<(int)grid_for(A.nnz, 256, kMaxGrid * 4), 256, 0, st>>>(A.nnz, A.ir, A.val,
                                                                                   ctx->aos.as<RowVal<V>>());
          arv = ctx->aos.as<RowVal<V>>();
        }
      }
      CAPCHK(cap);
      // tickets of the persistent kernels: sc[14], sc[15] (zeroed with the scalars)
      e = launch_num_heavy_known<CBG_KNOWN_LOGT, CBG_KNOWN_NT, SRT, V>(st, grid, known_list, sc + 12,
                                                                     A, B, spl, ou, sc + 14, arv);
      if (e == hipSuccess)
        e = launch_num_heavy<CBG_HEAVY_LOGT, CBG_HEAVY_NT, SRT, V>(st, grid, ctx->oitems.as<HeavyItem>(), sc + 13,
                                                                 ctx->heavy_cols.as<int32_t>(), units, nsub, A, B, span,
                                                                 spl, ou, sc + 15);
      HIPCHK(hipEventRecord(ctx->ev[7], st));
      // overflowed hash units -> single-subwindow (dense) units
      if (e == hipSuccess) {
        k_split_overflow_units<<<(int)grid_for(nunit_cap, 256, 1 << 20), 256, 0, st>>>(
            uovf_n, ctx->uovf_list.as<int32_t>(), units, ctx->sub.as<int32_t>(), nsub, ctx->fb_units.as<Unit>(), fb_n,
            ctx->fb_list.as<int32_t>());
        NumOut<V> of{own->ir.as<int32_t>(), own->val.as<V>(), adderr, fb_ovf_n, ctx->uovf_list.as<int32_t>()};
        e = launch_num_block<13, 1024, SRT, V, true>(st, ctx->fb_list.as<int32_t>(), fb_n, 0, 256,
                                                     ctx->fb_units.as<Unit>(), A, B, span, colptr, spl, of);
      }
    }
    // overflowed hash columns -> windowed dense sweep
    if (e == hipSuccess) {
      HIPCHK(ctx->cur.reserve(sizeof(int64_t) * (B.nnz + 1)));
      HIPCHK(ctx->nxt.reserve(sizeof(int32_t) * (B.nnz + 1)));
      CAPCHK(cap);
      e = launch_window<1, SRT, V, kWinRows>(st, ctx->ovf_list.as<int32_t>(), ovf_n, 0, 512, A, B, span, colptr,
                                             ctx->cur.as<int64_t>(), ctx->nxt.as<int32_t>(), nnz, ho, oc);
    }
    if (e != hipSuccess) { fprintf(stderr, "cbgpu: numeric launch: %s\n", hipGetErrorString(e)); return CBG_EDEVICE; }
    HIPCHK(hipGetLastError());
  }
  HIPCHK(hipEventRecord(ctx->ev[5], st));
  // the error ints (sc[2..5]), the rows-known unit count sc[12] and the heavy sums sc[16..18] (zero unless H > 0)
  HIPCHK(mirror(64, 64 + 19));
  HIPCHK(hipStreamSynchronize(st));
  const int* herr = (const int*)(psc + 2);
  const unsigned long long hknown = psc[12];
  const unsigned long long* hsum = psc + 16;
  float t;
  (void)hipEventElapsedTime(&t, ctx->ev[0], ctx->ev[1]); pf.flops_ms = t;
  (void)hipEventElapsedTime(&t, ctx->ev[1], ctx->ev[2]); pf.bin_ms = t;
  (void)hipEventElapsedTime(&t, ctx->ev[2], ctx->ev[3]); pf.symbolic_ms = t;
  (void)hipEventElapsedTime(&t, ctx->ev[3], ctx->ev[4]); pf.scan_ms = t;
  (void)hipEventElapsedTime(&t, ctx->ev[4], ctx->ev[5]); pf.numeric_ms = t;
  (void)hipEventElapsedTime(&t, ctx->ev[0], ctx->ev[5]); pf.total_ms = t;
  if (H > 0) { (void)hipEventElapsedTime(&t, ctx->ev[6], ctx->ev[7]); pf.heavy_ms = t; }
  pf.known_items = (int64_t)hknown;
  pf.heavy_multiplies = (int64_t)hsum[0];
  pf.heavy_nnz_b = (int64_t)hsum[1];
  pf.heavy_nnz_c = (int64_t)hsum[2];
  pf.bins[14] = herr[4];   // overflowed units (re-run dense per subwindow)
  pf.bins[15] = herr[3];   // overflowed columns (windowed fallback)
  C->nnz = nnzc;
  C->colptr = colptr;
  C->row = own->ir.as<int32_t>();
  C->val = own->val.p;
  C->multiplies = mults;
  C->_owner = own.release();
  if (mult_out) *mult_out = mults;
  if (herr[6]) {   // a fallback unit overflowed: only possible when SUBW > 8192 rows (nrow > 2^24)
    fprintf(stderr, "cbgpu: %d dense fallback units overflowed\n", herr[6]);
    return CBG_EUNSUP;
  }
  if (herr[2]) return CBG_EADD;
  return CBG_OK;
}

template <int SRI, typename V, bool MERGE>
using Pick = std::conditional_t<MERGE, MergeOf<Semiring<SRI, V>>, Semiring<SRI, V>>;

template <typename V, bool MERGE = false>
cbg_status dispatch_sr(cbg_ctx* ctx, const cbg_dcsc_view* A, const cbg_dcsc_view* B, cbg_semiring sr, uint32_t f,
                       cbg_csc_result* C, int64_t* m) {
  switch (sr) {
    case CBG_SR_PLUS_TIMES: return spgemm_impl<Pick<SR_PLUS_TIMES, V, MERGE>, V>(ctx, A, B, f, C, m);
    case CBG_SR_MIN_PLUS: return spgemm_impl<Pick<SR_MIN_PLUS, V, MERGE>, V>(ctx, A, B, f, C, m);
    case CBG_SR_SELECT2ND: return spgemm_impl<Pick<SR_SELECT2ND, V, MERGE>, V>(ctx, A, B, f, C, m);
    case CBG_SR_SELECT_MAX: return spgemm_impl<Pick<SR_SELECT_MAX, V, MERGE>, V>(ctx, A, B, f, C, m);
    case CBG_SR_SELECT_MAX_BOOL: return spgemm_impl<Pick<SR_SELECT_MAX_BOOL, V, MERGE>, V>(ctx, A, B, f, C, m);
    case CBG_SR_BOOL_COPY1ST: return spgemm_impl<Pick<SR_BOOL_COPY1ST, V, MERGE>, V>(ctx, A, B, f, C, m);
    case CBG_SR_BOOL_COPY2ND: return spgemm_impl<Pick<SR_BOOL_COPY2ND, V, MERGE>, V>(ctx, A, B, f, C, m);
  }
  return CBG_EUNSUP;
}

// concatenated partials: colptr[l*ncol + j] = off_l + cp_l[j]; selector: Sel(:, j) = {l*ncol + j}
static __global__ void k_merge_cat_cp(int64_t ncol, const int64_t* __restrict__ cp, int64_t off, int64_t* __restrict__ out) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < ncol; j += (int64_t)gridDim.x * blockDim.x)
    out[j] = off + cp[j];
}
static __global__ void k_merge_selector(int64_t ncol, int32_t k, int64_t* __restrict__ scp, int32_t* __restrict__ sir) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j <= ncol; j += (int64_t)gridDim.x * blockDim.x) {
    scp[j] = j * k;
    if (j < ncol)
      for (int32_t l = 0; l < k; ++l) sir[j * k + l] = (int32_t)(l * ncol + j);
  }
}

// ---- two-way merge of column-sorted partials (the 1x1x2 fiber merge, the q = 2 stage merges) ----
// One wave per column walks both sorted columns in windows of 64 merged positions: the window's rows
// are staged in LDS (pads: INT32_MAX), lane l finds merged position l by a merge-path search (ties take
// part 0 first, so a duplicate row is a (part 0, part 1) pair at adjacent positions), heads of equal-row
// runs are ranked by ballot, and a window never ends between the two halves of a pair.  Count pass ->
// nnz per column; fill pass -> rows and values at the scanned offsets.  Duplicates combine as
// MultiwayMergeHash does (MultiwayMerge.h:357, SR::add in part order): PlusTimes sums (bool: OR), MinPlus
// min, SelectMax max, Select2nd keeps part 0's value; BoolCopy1st/2nd count them as an error (CBG_EADD).
template <int SRI, typename V>
__device__ __forceinline__ V merge_pair(V a, V b) {
  if constexpr (SRI == SR_PLUS_TIMES) {
    if constexpr (sizeof(V) == 1) return (V)((a != 0) | (b != 0));
    else return a + b;
  } else if constexpr (SRI == SR_MIN_PLUS) {
    return b < a ? b : a;
  } else if constexpr (SRI == SR_SELECT_MAX || SRI == SR_SELECT_MAX_BOOL) {
    return b > a ? b : a;
  } else {
    return a;
  }
}

#ifndef CBG_MERGE_PL
#define CBG_MERGE_PL 4   // merged positions per lane per window (window = 64 * CBG_MERGE_PL)
#endif
// (staging the fill pass's values and merged output in LDS for coalesced loads/stores measured slower: s22 rank share
// 85.7 vs 67.8 ms, 24 KB of LDS per block; removed in round 6)
constexpr int kMergePL = CBG_MERGE_PL;
constexpr int kMergeW = kWave * kMergePL;
static_assert(kMergeW < 1024, "the merge window's counts are packed in 10-bit fields");

template <int SRI, typename V, bool FILL>
__global__ void __launch_bounds__(256) k_merge2(int64_t ncol, const int64_t* __restrict__ acp,
                                                const int32_t* __restrict__ air, const V* __restrict__ aval,
                                                const int64_t* __restrict__ bcp, const int32_t* __restrict__ bir,
                                                const V* __restrict__ bval, int64_t* __restrict__ cnt,
                                                const int64_t* __restrict__ ccp, int32_t* __restrict__ crow,
                                                V* __restrict__ cval, unsigned long long* __restrict__ dups,
                                                unsigned long long* __restrict__ disorder) {
  constexpr int W = kMergeW, PL = kMergePL;
  __shared__ int32_t swin[4][2][W];
  const int w = threadIdx.x / kWave, l = lane_id();
  int32_t* sa = swin[w][0];
  int32_t* sb = swin[w][1];
  for (int64_t j = (int64_t)blockIdx.x * 4 + w; j < ncol; j += (int64_t)gridDim.x * 4) {
    int64_t ia = acp[j], ib = bcp[j];
    const int64_t ea = acp[j + 1], eb = bcp[j + 1];
    int64_t o = FILL ? ccp[j] : 0;
    unsigned long long nd = 0, bad = 0;
    const int64_t a0 = ia, b0 = ib;
    while (ia < ea || ib < eb) {   // wave-uniform
#pragma unroll
      for (int r = 0; r < PL; ++r) {
        const int x = l + r * kWave;
        sa[x] = ia + x < ea ? air[ia + x] : INT32_MAX;
        sb[x] = ib + x < eb ? bir[ib + x] : INT32_MAX;
      }
      wave_sync();
      if (!FILL) {   // the merge needs strictly ascending rows per column: verify in the count pass
#pragma unroll
        for (int r = 0; r < PL; ++r) {
          const int x = l + r * kWave;
          const int32_t pa = x > 0 ? sa[x - 1] : (ia > a0 ? air[ia - 1] : -1);
          const int32_t pb = x > 0 ? sb[x - 1] : (ib > b0 ? bir[ib - 1] : -1);
          bad += (ia + x < ea && sa[x] <= pa) || (ib + x < eb && sb[x] <= pb);
        }
      }
      // this lane's merged positions d0 .. d0+PL-1; split at d0 by a merge-path search (ties: part 0 first)
      const int d0 = l * PL;
      int lo = d0 > W ? d0 - W : 0, hi = d0 < W ? d0 : W;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (sa[mid] <= sb[d0 - 1 - mid]) lo = mid + 1; else hi = mid;
      }
      int i = lo, jb = d0 - lo;
      int32_t row[PL];
      int src[PL];            // part-0 index, or -1 - part-1 index
      bool pair[PL];
#pragma unroll
      for (int e = 0; e < PL; ++e) {
        const bool take_a = i < W && (jb >= W || sa[i] <= sb[jb]);
        row[e] = take_a ? sa[i] : sb[jb];
        pair[e] = take_a && row[e] != INT32_MAX && jb < W && sb[jb] == row[e];
        src[e] = take_a ? i : -1 - jb;
        if (take_a) ++i; else ++jb;
      }
      // a pair must not straddle windows: the window ends before the last position if it is a part-0 half
      const int K = __shfl(pair[PL - 1] ? W - 1 : W, kWave - 1, kWave);
      int32_t prev = __shfl_up(row[PL - 1], 1, kWave);
      int c = 0, na = 0;
      bool head[PL];
#pragma unroll
      for (int e = 0; e < PL; ++e) {
        const bool in = d0 + e < K && row[e] != INT32_MAX;
        head[e] = in && ((d0 + e == 0) || prev != row[e]);
        prev = row[e];
        c += head[e];
        na += in && src[e] >= 0;
        if (!FILL && in && pair[e]) ++nd;
      }
      int nin = 0;
#pragma unroll
      for (int e = 0; e < PL; ++e) nin += d0 + e < K && row[e] != INT32_MAX;
      // one wave scan for the three window counts (each <= W < 1024): heads | part-0 taken << 10 | in window << 20
      const int pk = wave_incl_scan(c | (na << 10) | (nin << 20));
      const int incl = pk & 1023;
      const int ptot = __shfl(pk, kWave - 1, kWave);
      const int tot = ptot & 1023, ta = (ptot >> 10) & 1023, tin = ptot >> 20;
      if (FILL) {
        int64_t pos = o + incl - c;
#pragma unroll
        for (int e = 0; e < PL; ++e)
          if (head[e]) {
            const int s = src[e];
            V v = s >= 0 ? (aval ? aval[ia + s] : V(1)) : (bval ? bval[ib + (-1 - s)] : V(1));
            if (pair[e]) v = merge_pair<SRI, V>(v, bval ? bval[ib + d0 + e - s] : V(1));
            crow[pos] = row[e];
            cval[pos] = v;
            ++pos;
          }
      }
      o += tot;
      ia += ta;
      ib += tin - ta;
      wave_sync();
    }
    if (!FILL) {
      const unsigned long long d = (unsigned long long)wave_sum64((int64_t)nd);
      const unsigned long long x = (unsigned long long)wave_sum64((int64_t)bad);
      if (l == 0) {
        cnt[j] = o;
        if (d) atomicAdd(dups, d);
        if (x) atomicAdd(disorder, x);
      }
    }
  }
}

// ---- flat two-way merge (default; CBG_MERGE_FLAT=0 takes the per-column k_merge2 above) ----
// The merged sequence of both partials -- keys (column, row), duplicates kept, column c starting at merged position
// acp[c] + bcp[c] -- is cut into tiles of kFlatT positions regardless of column lengths, so every workgroup moves
// the same number of entries: one 330k-position column is ~320 tiles, a run of short columns shares one tile.
// k_flat_split finds each tile boundary (binary search over the column starts, then a merge-path search inside the
// column) and moves it one position back when it would separate a (part 0, part 1) pair of equal keys.  A tile
// stages both of its key runs in LDS -- the column of every entry from the column starts inside the tile (marks +
// a block max-scan) -- each thread takes kFlatPT merged positions by a merge-path search, heads of equal-key runs
// are counted (count pass) or written at the scanned offsets with the column pointers that start inside the tile
// (fill pass).  The count pass reads rows only; the fill pass reads rows and values once and writes C once.
// tile boundaries every kFlatT = kFlatNT * kFlatPT - 1 positions: a boundary moved back by a pair makes its tile one
// position longer, so a tile holds at most kFlatNT * kFlatPT positions -- one per thread slot
constexpr int kFlatNT = 256, kFlatPT = 4, kFlatT = kFlatNT * kFlatPT - 1;
constexpr int kFlatCH = (kFlatT + 2 + kFlatNT - 1) / kFlatNT;   // staged entries per thread in the column scan

static __global__ void k_flat_split(int64_t ncol, const int64_t* __restrict__ acp, const int32_t* __restrict__ air,
                             const int64_t* __restrict__ bcp, const int32_t* __restrict__ bir, int64_t ntiles,
                             int64_t* __restrict__ sa, int64_t* __restrict__ sb, int32_t* __restrict__ sc) {
  const int64_t na = acp[ncol], nb = bcp[ncol], dt = na + nb;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t <= ntiles; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t d = t * kFlatT;
    if (d >= dt) {
      sa[t] = na; sb[t] = nb; sc[t] = (int32_t)ncol;
      continue;
    }
    int64_t lo = 0, hi = ncol - 1;   // the last column starting at or before d (it holds position d)
    while (lo < hi) {
      const int64_t mid = (lo + hi + 1) >> 1;
      if (acp[mid] + bcp[mid] <= d) lo = mid; else hi = mid - 1;
    }
    const int64_t c = lo, ca = acp[c], cb = bcp[c];
    const int64_t la = acp[c + 1] - ca, lb = bcp[c + 1] - cb, k = d - ca - cb;
    int64_t i0 = k > lb ? k - lb : 0, i1 = k < la ? k : la;
    while (i0 < i1) {   // part-0 entries among the column's first k merged positions (ties: part 0 first)
      const int64_t mid = (i0 + i1) >> 1;
      if (air[ca + mid] <= bir[cb + k - 1 - mid]) i0 = mid + 1; else i1 = mid;
    }
    int64_t i = i0;
    const int64_t j = k - i;
    if (i > 0 && j < lb && air[ca + i - 1] == bir[cb + j]) --i;   // keep the pair together
    sa[t] = ca + i; sb[t] = cb + j; sc[t] = (int32_t)c;
  }
}

__device__ __forceinline__ int wave_incl_max(int v) {
  const int l = lane_id();
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const int t = __shfl_up(v, d, kWave);
    if (l >= d) v = max(v, t);
  }
  return v;
}

// col[x] = max(col[0..x]) over the staged part-0 run col[0..na) and, separately, the part-1 run cb[0..nb)
// (column starts were marked at their first entry); two barriers for both runs
__device__ __forceinline__ void block_col_scan2(int32_t* ca, int na, int32_t* cb, int nb, int* scratch) {
  constexpr int NW = kFlatNT / kWave;
  const int x0 = threadIdx.x * kFlatCH, w = threadIdx.x / kWave, l = lane_id();
  int ma = INT_MIN, mb = INT_MIN;
#pragma unroll
  for (int e = 0; e < kFlatCH; ++e) {
    if (x0 + e < na) ma = max(ma, ca[x0 + e]);
    if (x0 + e < nb) mb = max(mb, cb[x0 + e]);
  }
  const int ia = wave_incl_max(ma), ib = wave_incl_max(mb);
  if (l == kWave - 1) {
    scratch[w] = ia;
    scratch[NW + w] = ib;
  }
  __syncthreads();
  int ra = __shfl_up(ia, 1, kWave), rb = __shfl_up(ib, 1, kWave);
  if (l == 0) ra = rb = INT_MIN;
  for (int q = 0; q < w; ++q) {
    ra = max(ra, scratch[q]);
    rb = max(rb, scratch[NW + q]);
  }
#pragma unroll
  for (int e = 0; e < kFlatCH; ++e) {
    if (x0 + e < na) {
      ra = max(ra, ca[x0 + e]);
      ca[x0 + e] = ra;
    }
    if (x0 + e < nb) {
      rb = max(rb, cb[x0 + e]);
      cb[x0 + e] = rb;
    }
  }
  __syncthreads();
}

// tile prefix states of the one-pass merge: flag (bits 62-63) | value; flag 1 = the tile's count, 2 = inclusive prefix
// MODE 0: count pass (cnt[t] = heads of tile t); MODE 1: fill pass at the scanned offsets toff[t].  (A one-pass
// variant -- tiles claimed in order, offsets by a decoupled look-back -- measured 146 ms against 36.7 for the two
// passes at s20: the look-back chain serialises the tiles; staging the values in LDS too: 42.4 ms, r04k.)
// PF: the next tile's rows (and the starts of the columns inside it) are loaded into registers while the current tile
// merges, so a tile's chain is boundaries -> LDS -> merge path instead of boundaries -> rows -> LDS -> merge path.
template <int SRI, typename V, int MODE, bool PF>
__global__ void __launch_bounds__(kFlatNT) __attribute__((amdgpu_waves_per_eu(8, 8))) k_flat_merge(
    int64_t ncol, const int64_t* __restrict__ acp, const int32_t* __restrict__ air, const V* __restrict__ aval,
    const int64_t* __restrict__ bcp, const int32_t* __restrict__ bir, const V* __restrict__ bval,
    const int64_t* __restrict__ sa, const int64_t* __restrict__ sb, const int32_t* __restrict__ sc, int64_t ntiles,
    int64_t* __restrict__ cnt, const int64_t* __restrict__ toff, int64_t* __restrict__ ccp,
    int32_t* __restrict__ crow, V* __restrict__ cval, unsigned long long* __restrict__ dups,
    unsigned long long* __restrict__ disorder, bool stage_out) {
  constexpr bool FILL = MODE != 0;
  constexpr int T = kFlatT, PT = kFlatPT, NT = kFlatNT;
  static_assert(NT * PT >= T + 1, "every position of a tile has a thread slot");
  static_assert(NT * PT <= 32767, "16-bit head positions");
  // one key array for both runs: part 0 at [0, na), a sentinel, part 1 at [na + 1, n + 1), a sentinel -- 14 KB of
  // LDS per workgroup, so 8 workgroups (the wave limit) fit a CU
  __shared__ uint64_t keys[T + 4];
  __shared__ int32_t cols[T + 4];
  __shared__ int16_t hpos[T + 2];
  __shared__ int scr[2 * (NT / kWave) + 2];
  const int tid = threadIdx.x;
  unsigned long long bad = 0, ndup = 0;   // summed over the block's tiles, one atomic per wave at the end
  int64_t t = blockIdx.x;
  int64_t a0 = 0, b0 = 0, a1 = 0, b1 = 0;
  int32_t c0 = 0, ce = 0;
  if (t < ntiles) {
    a0 = sa[t]; a1 = sa[t + 1]; b0 = sb[t]; b1 = sb[t + 1]; c0 = sc[t]; ce = sc[t + 1];
  }
  constexpr int KX = (T + 1 + NT - 1) / NT;   // tile entries per thread (both runs together hold <= T + 1)
  int32_t xr[KX];   // PF: row of tile entry y = tid + k*NT (part 0 at y < na, part 1 at y - na)
  auto fetch = [&](int64_t A0, int64_t A1, int64_t B0, int64_t B1) {
    const int64_t la = A1 - A0, lb = B1 - B0;
    const bool okt = la >= 0 && lb >= 0 && la + lb <= T + 1;
    const int fa = okt ? (int)la : 0, fn = okt ? (int)(la + lb) : 0;
#pragma unroll
    for (int k = 0; k < KX; ++k) {
      const int y = tid + k * NT;
      xr[k] = y < fa ? air[A0 + y] : y < fn ? bir[B0 + (y - fa)] : 0;
    }
  };
  if (PF && t < ntiles) fetch(a0, a1, b0, b1);
  while (t < ntiles) {
    // the next tile's boundaries, loaded while this one is merged
    const int64_t tn = t + gridDim.x;
    int64_t na0 = 0, nb0 = 0, na1 = 0, nb1 = 0;
    int32_t nc0 = 0, nce = 0;
    if (tn < ntiles) {
      na0 = sa[tn]; na1 = sa[tn + 1]; nb0 = sb[tn]; nb1 = sb[tn + 1]; nc0 = sc[tn]; nce = sc[tn + 1];
    }
    const int64_t ta = a1 - a0, tb = b1 - b0;
    if (ta < 0 || tb < 0 || ta + tb > T + 1) {   // boundaries out of order: only a partial with unsorted rows
      if (!FILL && tid == 0) {
        cnt[t] = 0;
        ++bad;
      }
      if (PF && tn < ntiles) fetch(na0, na1, nb0, nb1);
    } else {
      const int na = (int)ta, nb = (int)tb, n = na + nb;
      uint64_t* ka = keys;
      uint64_t* kb = keys + na + 1;
      int32_t* ca = cols;
      int32_t* cb = cols + na + 1;
      // a column boundary inside the tile?  (uniform) -- tiles inside one long column skip the column scan
      const int32_t cl = ce < ncol ? ce : (int32_t)(ncol - 1);
      const bool multi = cl > c0;
      // tile-edge order check: the entry before each run, when it lies in the run's first column
      int32_t pra = -1, prb = -1;
      int64_t acp0 = 0, bcp0 = 0;
      if (!FILL && tid == 0) {
        acp0 = acp[c0]; bcp0 = bcp[c0];
        if (a0 > 0) pra = air[a0 - 1];
        if (b0 > 0) prb = bir[b0 - 1];
      }
      if (multi) {
        for (int x = tid; x < na; x += NT) ca[x] = c0;
        for (int x = tid; x < nb; x += NT) cb[x] = c0;
        __syncthreads();
        for (int64_t c = (int64_t)c0 + 1 + tid; c <= cl; c += NT) {   // columns starting inside the tile
          const int64_t pa = acp[c] - a0, pb = bcp[c] - b0;
          if (pa < na) atomicMax(&ca[pa], (int)c);
          if (pb < nb) atomicMax(&cb[pb], (int)c);
        }
        __syncthreads();
        block_col_scan2(ca, na, cb, nb, scr);
      }
      if (PF) {
#pragma unroll
        for (int k = 0; k < KX; ++k) {   // keys[] holds part 0 at [0, na), part 1 at [na + 1, n + 1)
          const int y = tid + k * NT;
          if (y < n) {
            const int32_t cy = multi ? (y < na ? ca[y] : cb[y - na]) : c0;
            keys[y < na ? y : y + 1] = ((uint64_t)(uint32_t)cy << 32) | (uint32_t)xr[k];
          }
        }
        if (tn < ntiles) fetch(na0, na1, nb0, nb1);   // in flight while this tile merges
      } else {
        for (int x = tid; x < na; x += NT)
          ka[x] = ((uint64_t)(uint32_t)(multi ? ca[x] : c0) << 32) | (uint32_t)air[a0 + x];
        for (int x = tid; x < nb; x += NT)
          kb[x] = ((uint64_t)(uint32_t)(multi ? cb[x] : c0) << 32) | (uint32_t)bir[b0 + x];
      }
      if (tid == 0) {
        ka[na] = ~0ull;
        kb[nb] = ~0ull;
      }
      __syncthreads();
      if (!FILL) {   // the merge needs strictly ascending rows per column
        for (int x = tid + 1; x < na; x += NT) bad += ka[x] <= ka[x - 1];
        for (int x = tid + 1; x < nb; x += NT) bad += kb[x] <= kb[x - 1];
        if (tid == 0) {
          if (na > 0 && (uint32_t)(ka[0] >> 32) == (uint32_t)c0 && a0 > acp0) bad += (uint32_t)ka[0] <= (uint32_t)pra;
          if (nb > 0 && (uint32_t)(kb[0] >> 32) == (uint32_t)c0 && b0 > bcp0) bad += (uint32_t)kb[0] <= (uint32_t)prb;
        }
      }
      // this thread's merged positions d0 .. d0+PT-1
      const int d0 = tid * PT;
      int lo = d0 > nb ? d0 - nb : 0, hi = d0 < na ? d0 : na;
      if (d0 > n) lo = hi = 0;   // idle thread (n < T): no position, no reads
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (ka[mid] <= kb[d0 - 1 - mid]) lo = mid + 1; else hi = mid;
      }
      int i = lo, j = d0 - lo;
      // key at position d0 - 1: the larger of the last part-0 and part-1 keys taken so far
      uint64_t prev = 0;
      bool has_prev = d0 > 0 && d0 <= n;
      if (has_prev) {
        const uint64_t pa = i > 0 ? ka[i - 1] : 0, pb = j > 0 ? kb[j - 1] : 0;
        prev = pa > pb ? pa : pb;
      }
      uint32_t row[PT];
      int src[PT];   // part-0 index, or -1 - part-1 index
      bool head[PT], pair[PT];
      int c = 0, nd = 0;
#pragma unroll
      for (int e = 0; e < PT; ++e) {
        const bool in = d0 + e < n;   // then i < na or j < nb
        const bool take_a = in && i < na && (j >= nb || ka[i] <= kb[j]);
        const uint64_t key = !in ? ~0ull : take_a ? ka[i] : kb[j];
        row[e] = (uint32_t)key;
        src[e] = take_a ? i : -1 - j;
        pair[e] = take_a && j < nb && kb[j] == key;
        head[e] = in && (!has_prev || key != prev);
        has_prev = true;
        prev = key;
        if (in) { if (take_a) ++i; else ++j; }
        c += head[e];
        nd += pair[e];
      }
      if (!FILL) {
        int tot;
        (void)block_excl_scan<NT>(c, scr, &tot);
        ndup += nd;
        if (tid == 0) cnt[t] = tot;
      } else {
        V v[PT];   // the values are gathered before the scan's barriers
#pragma unroll
        for (int e = 0; e < PT; ++e) {
          v[e] = V(0);
          if (head[e]) {
            const int s = src[e];
            v[e] = s >= 0 ? (aval ? aval[a0 + s] : V(1)) : (bval ? bval[b0 + (-1 - s)] : V(1));
            if (pair[e]) v[e] = merge_pair<SRI, V>(v[e], bval ? bval[b0 + (d0 + e - s)] : V(1));
          }
        }
        int tot;
        const int ex = block_excl_scan<NT>(c, scr, &tot);   // its barriers also end every read of keys / cols
        const int64_t o = toff[t];
        int q = ex;
        if (stage_out) {   // the tile's output through LDS (over the staged keys): coalesced stores
          int32_t* orow = cols;
          V* oval = (V*)keys;
#pragma unroll
          for (int e = 0; e < PT; ++e) {
            if (d0 + e < n) hpos[d0 + e] = (int16_t)q;
            if (head[e]) {
              orow[q] = (int32_t)row[e];
              oval[q] = v[e];
              ++q;
            }
          }
          if (tid == 0) hpos[n] = (int16_t)tot;
          __syncthreads();
          for (int x = tid; x < tot; x += NT) {
            crow[o + x] = orow[x];
            cval[o + x] = oval[x];
          }
        } else {
#pragma unroll
          for (int e = 0; e < PT; ++e) {
            if (d0 + e < n) hpos[d0 + e] = (int16_t)q;
            if (head[e]) {
              crow[o + q] = (int32_t)row[e];
              cval[o + q] = v[e];
              ++q;
            }
          }
          if (tid == 0) hpos[n] = (int16_t)tot;
          __syncthreads();
        }
        // column pointers of the columns starting in this tile (a column starting exactly at the tile's end is
        // written by both neighbours, with the same value); tile 0 also owns the empty columns before c0
        const int64_t dbase = a0 + b0;
        const int64_t cs = t == 0 ? 0 : c0, cend = ce < ncol ? ce : ncol;
        for (int64_t cc = cs + tid; cc <= cend; cc += NT) {
          const int64_t dl = acp[cc] + bcp[cc] - dbase;
          if (dl >= 0 && dl <= n) ccp[cc] = o + hpos[dl];
        }
      }
    }
    __syncthreads();   // the tile's LDS is free for the next one
    t = tn;
    a0 = na0; a1 = na1; b0 = nb0; b1 = nb1; c0 = nc0; ce = nce;
  }
  if (!FILL) {
    const int64_t d = wave_sum64((int64_t)ndup), x = wave_sum64((int64_t)bad);
    if (lane_id() == 0) {
      if (d) atomicAdd(dups, (unsigned long long)d);
      if (x) atomicAdd(disorder, (unsigned long long)x);
    }
  }
}

template <int SRI, typename V>
cbg_status merge2_flat(cbg_ctx* ctx, const cbg_csc_result* parts, cbg_csc_result* C) {
  hipStream_t st = ctx->stream;
  const int64_t ncol = parts[0].ncol;
  const bool add_is_error = SRI == SR_BOOL_COPY1ST || SRI == SR_BOOL_COPY2ND;
  const int64_t dt = parts[0].nnz + parts[1].nnz;
  const char* se = std::getenv("CBG_MERGE_STAGE");   // 0: the fill pass stores from registers
  const bool stage = !se || std::atoi(se) != 0;
  // row prefetch (k_flat_merge PF) in both passes (s20 1x1x2 partials: 36.8 -> 31.7 ms, profiles/r05b_merge_pf.txt,
  // although the fill pass spills one register at 8 waves per SIMD); CBG_MERGE_PF=1 count pass only, 0 neither
  static const int pfm = [] { const char* x = std::getenv("CBG_MERGE_PF"); return x ? std::atoi(x) : 2; }();
  const bool pf = pfm >= 1, pf_fill = pfm >= 2;
  if (ncol >= INT32_MAX) return CBG_EINVAL;   // the staged keys carry 32-bit columns: the per-column merge runs
  std::unique_ptr<Owner> own(new Owner(ctx->pool));
  HIPCHK(own->cp.reserve(8 * (ncol + 1)));
  const V* av = (const V*)parts[0].val;
  const V* bv = (const V*)parts[1].val;
  int64_t nnz = 0;
  if (ncol == 0 || dt == 0) {
    HIPCHK(hipMemsetAsync(own->cp.p, 0, 8 * (ncol + 1), st));
    HIPCHK(own->ir.reserve(4));
    HIPCHK(own->val.reserve(sizeof(V)));
    HIPCHK(hipStreamSynchronize(st));
  } else {
    const int64_t ntiles = (dt + kFlatT - 1) / kFlatT;
    PoolBuf cnt, tiles, spl;
    cnt.pool = tiles.pool = spl.pool = ctx->pool;
    HIPCHK(spl.reserve(20 * (ntiles + 1) + 16));
    HIPCHK(cnt.reserve(16 * (ntiles + 1)));   // tile counts, then their exclusive offsets
    int64_t* toff = cnt.as<int64_t>() + ntiles + 1;
    const int64_t nst = (ntiles + kScanTile - 1) / kScanTile;
    HIPCHK(tiles.reserve(8 * (nst + 1)));
    HIPCHK(ctx->scalars.reserve(256));
    unsigned long long* sc = ctx->scalars.as<unsigned long long>();
    HIPCHK(hipMemsetAsync(sc, 0, 24, st));
    int64_t* sa = spl.as<int64_t>();
    int64_t* sb = sa + ntiles + 1;
    int32_t* scol = (int32_t*)(sb + ntiles + 1);
    k_flat_split<<<(int)grid_for(ntiles + 1, 256, kMaxGrid * 4), 256, 0, st>>>(
        ncol, parts[0].colptr, parts[0].row, parts[1].colptr, parts[1].row, ntiles, sa, sb, scol);
    const int g = (int)grid_for(ntiles, 1, kMaxGrid * 8);
    unsigned long long* h = pinned<unsigned long long>(ctx, kPinMerge);   // pairs, nnz(C), disorder
    if (pf)
      k_flat_merge<SRI, V, 0, true><<<g, kFlatNT, 0, st>>>(ncol, parts[0].colptr, parts[0].row, av, parts[1].colptr,
                                                         parts[1].row, bv, sa, sb, scol, ntiles, cnt.as<int64_t>(),
                                                         nullptr, nullptr, nullptr, nullptr, sc, sc + 2, false);
    else
      k_flat_merge<SRI, V, 0, false><<<g, kFlatNT, 0, st>>>(ncol, parts[0].colptr, parts[0].row, av, parts[1].colptr,
                                                          parts[1].row, bv, sa, sb, scol, ntiles, cnt.as<int64_t>(),
                                                          nullptr, nullptr, nullptr, nullptr, sc, sc + 2, false);
    k_scan_tiles<<<(int)nst, 256, 0, st>>>(ntiles, cnt.as<int64_t>(), tiles.as<int64_t>());
    k_scan_sums<<<1, 1024, 0, st>>>(nst, tiles.as<int64_t>(), (int64_t*)(sc + 1));
    k_scan_apply<<<(int)nst, 256, 0, st>>>(ntiles, cnt.as<int64_t>(), tiles.as<int64_t>(), toff);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(h, sc, 24, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (h[2]) return CBG_EINVAL;   // a partial is not row-sorted: the caller takes the hash merge
    if (add_is_error && h[0]) return CBG_EADD;
    nnz = (int64_t)h[1];
    if (own->ir.reserve(4 * (nnz + 1)) != hipSuccess || own->val.reserve(sizeof(V) * (nnz + 1)) != hipSuccess) {
      (void)hipGetLastError();
      release_workspace(ctx);
      HIPCHK(own->ir.reserve(4 * (nnz + 1)));
      HIPCHK(own->val.reserve(sizeof(V) * (nnz + 1)));
    }
    if (pf_fill)
      k_flat_merge<SRI, V, 1, true><<<g, kFlatNT, 0, st>>>(ncol, parts[0].colptr, parts[0].row, av, parts[1].colptr,
                                                         parts[1].row, bv, sa, sb, scol, ntiles, nullptr, toff,
                                                         own->cp.as<int64_t>(), own->ir.as<int32_t>(), own->val.as<V>(),
                                                         nullptr, nullptr, stage);
    else
      k_flat_merge<SRI, V, 1, false><<<g, kFlatNT, 0, st>>>(ncol, parts[0].colptr, parts[0].row, av, parts[1].colptr,
                                                          parts[1].row, bv, sa, sb, scol, ntiles, nullptr, toff,
                                                          own->cp.as<int64_t>(), own->ir.as<int32_t>(),
                                                          own->val.as<V>(), nullptr, nullptr, stage);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(st));   // split / cnt / tiles go back to the pool on return
  }
  memset(C, 0, sizeof(*C));
  C->nrow = parts[0].nrow; C->ncol = ncol; C->nnz = nnz;
  C->colptr = own->cp.as<int64_t>(); C->row = own->ir.as<int32_t>(); C->val = own->val.p;
  C->val_type = DtOf<V>::value;
  C->_owner = own.release();
  return CBG_OK;
}

template <int SRI, typename V>
cbg_status merge2_sr(cbg_ctx* ctx, const cbg_csc_result* parts, cbg_csc_result* C) {
  const char* fe = std::getenv("CBG_MERGE_FLAT");
  const bool flat = !fe || std::atoi(fe) != 0;
  if (flat && parts[0].ncol < INT32_MAX) return merge2_flat<SRI, V>(ctx, parts, C);
  hipStream_t st = ctx->stream;
  const int64_t ncol = parts[0].ncol;
  const bool add_is_error = SRI == SR_BOOL_COPY1ST || SRI == SR_BOOL_COPY2ND;
  std::unique_ptr<Owner> own(new Owner(ctx->pool));
  PoolBuf cnt, tiles;
  cnt.pool = tiles.pool = ctx->pool;
  HIPCHK(own->cp.reserve(8 * (ncol + 1)));
  HIPCHK(cnt.reserve(8 * (ncol + 1)));
  const int64_t ntiles = (ncol + kScanTile - 1) / kScanTile;
  HIPCHK(tiles.reserve(8 * (ntiles + 1)));
  HIPCHK(ctx->scalars.reserve(256));
  unsigned long long* sc = ctx->scalars.as<unsigned long long>();
  HIPCHK(hipMemsetAsync(sc, 0, 24, st));
  const int g = (int)grid_for(ncol, 4, kMaxGrid * 8);
  const V* av = (const V*)parts[0].val;
  const V* bv = (const V*)parts[1].val;
  k_merge2<SRI, V, false><<<g, 256, 0, st>>>(ncol, parts[0].colptr, parts[0].row, av, parts[1].colptr, parts[1].row,
                                             bv, cnt.as<int64_t>(), nullptr, nullptr, nullptr, sc, sc + 2);
  if (ncol > 0) {
    k_scan_tiles<<<(int)ntiles, 256, 0, st>>>(ncol, cnt.as<int64_t>(), tiles.as<int64_t>());
    k_scan_sums<<<1, 1024, 0, st>>>(ntiles, tiles.as<int64_t>(), (int64_t*)(sc + 1));
    k_scan_apply<<<(int)ntiles, 256, 0, st>>>(ncol, cnt.as<int64_t>(), tiles.as<int64_t>(), own->cp.as<int64_t>());
  } else {
    HIPCHK(hipMemsetAsync(own->cp.p, 0, 8, st));
  }
  HIPCHK(hipGetLastError());
  unsigned long long* h = pinned<unsigned long long>(ctx, kPinMerge);   // duplicate pairs, nnz(C), columns out of order
  HIPCHK(hipMemcpyAsync(h, sc, 24, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (h[2]) return CBG_EINVAL;   // a partial is not row-sorted: the caller takes the hash merge
  if (add_is_error && h[0]) return CBG_EADD;   // BoolCopy add() would have been called (it throws)
  const int64_t nnz = (int64_t)h[1];
  if (own->ir.reserve(4 * (nnz + 1)) != hipSuccess || own->val.reserve(sizeof(V) * (nnz + 1)) != hipSuccess) {
    (void)hipGetLastError();
    release_workspace(ctx);   // the product workspace is idle between calls: give it back and retry once
    HIPCHK(own->ir.reserve(4 * (nnz + 1)));
    HIPCHK(own->val.reserve(sizeof(V) * (nnz + 1)));
  }
  k_merge2<SRI, V, true><<<g, 256, 0, st>>>(ncol, parts[0].colptr, parts[0].row, av, parts[1].colptr, parts[1].row, bv,
                                            nullptr, own->cp.as<int64_t>(), own->ir.as<int32_t>(), own->val.as<V>(),
                                            nullptr, nullptr);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(st));   // cnt / tiles go back to the pool on return
  memset(C, 0, sizeof(*C));
  C->nrow = parts[0].nrow; C->ncol = ncol; C->nnz = nnz;
  C->colptr = own->cp.as<int64_t>(); C->row = own->ir.as<int32_t>(); C->val = own->val.p;
  C->val_type = DtOf<V>::value;
  C->_owner = own.release();
  return CBG_OK;
}

template <typename V>
cbg_status merge2(cbg_ctx* ctx, const cbg_csc_result* parts, cbg_semiring sr, cbg_csc_result* C) {
  switch (sr) {
    case CBG_SR_PLUS_TIMES: return merge2_sr<SR_PLUS_TIMES, V>(ctx, parts, C);
    case CBG_SR_MIN_PLUS: return merge2_sr<SR_MIN_PLUS, V>(ctx, parts, C);
    case CBG_SR_SELECT2ND: return merge2_sr<SR_SELECT2ND, V>(ctx, parts, C);
    case CBG_SR_SELECT_MAX: return merge2_sr<SR_SELECT_MAX, V>(ctx, parts, C);
    case CBG_SR_SELECT_MAX_BOOL: return merge2_sr<SR_SELECT_MAX_BOOL, V>(ctx, parts, C);
    case CBG_SR_BOOL_COPY1ST: return merge2_sr<SR_BOOL_COPY1ST, V>(ctx, parts, C);
    case CBG_SR_BOOL_COPY2ND: return merge2_sr<SR_BOOL_COPY2ND, V>(ctx, parts, C);
  }
  return CBG_EUNSUP;
}

template <typename V>
cbg_status merge_impl(cbg_ctx* ctx, const cbg_csc_result* parts, int32_t k, cbg_semiring sr, uint32_t flags,
                      cbg_csc_result* C) {
  const int64_t nrow = parts[0].nrow, ncol = parts[0].ncol;
  int64_t tot = 0;
  for (int32_t l = 0; l < k; ++l) {
    if (parts[l].nrow != nrow || parts[l].ncol != ncol) return CBG_EDIM;   // MultiwayMerge.h:443-450
    if (parts[l].val_type != DtOf<V>::value) return CBG_EINVAL;
    tot += parts[l].nnz;
  }
  // two partials (every mandated layout's merges): the dedicated two-way merge; it verifies that the
  // partials' columns are row-sorted and declines (CBG_EINVAL) otherwise, then the hash merge below runs
  if (k == 2 && std::getenv("CBG_MERGE_PRODUCT") == nullptr) {
    const cbg_status s2 = merge2<V>(ctx, parts, sr, C);
    if (s2 != CBG_EINVAL) return s2;
  }
  if ((int64_t)k * ncol >= INT32_MAX) return CBG_EUNSUP;
  hipStream_t st = ctx->stream;
  // scratch from the context's caching pool (a fresh hipMalloc/hipFree pair per merge costs more than a
  // small merge; hipFree also synchronises the device)
  PoolBuf cat_cp, cat_ir, cat_val, sel_cp, sel_ir;
  cat_cp.pool = cat_ir.pool = cat_val.pool = sel_cp.pool = sel_ir.pool = ctx->pool;
  HIPCHK(cat_cp.reserve(sizeof(int64_t) * (k * ncol + 1)));
  HIPCHK(cat_ir.reserve(sizeof(int32_t) * (tot + 1)));
  HIPCHK(cat_val.reserve(sizeof(V) * (tot + 1)));
  HIPCHK(sel_cp.reserve(sizeof(int64_t) * (ncol + 1)));
  HIPCHK(sel_ir.reserve(sizeof(int32_t) * (k * ncol + 1)));
  int64_t off = 0;
  for (int32_t l = 0; l < k; ++l) {
    const int64_t n = parts[l].nnz;
    if (n) {
      HIPCHK(hipMemcpyAsync(cat_ir.as<int32_t>() + off, parts[l].row, sizeof(int32_t) * n, hipMemcpyDeviceToDevice, st));
      HIPCHK(hipMemcpyAsync(cat_val.as<V>() + off, parts[l].val, sizeof(V) * n, hipMemcpyDeviceToDevice, st));
    }
    k_merge_cat_cp<<<(int)grid_for(ncol, 256, kMaxGrid), 256, 0, st>>>(ncol, parts[l].colptr, off,
                                                                      cat_cp.as<int64_t>() + l * ncol);
    off += n;
  }
  HIPCHK(hipMemcpyAsync(cat_cp.as<int64_t>() + (int64_t)k * ncol, &tot, sizeof(int64_t), hipMemcpyHostToDevice, st));
  k_merge_selector<<<(int)grid_for(ncol + 1, 256, kMaxGrid), 256, 0, st>>>(ncol, k, sel_cp.as<int64_t>(),
                                                                           sel_ir.as<int32_t>());
  HIPCHK(hipGetLastError());
  cbg_dcsc_view a{}, b{};
  a.nrow = nrow; a.ncol = (int64_t)k * ncol; a.nnz = tot; a.nzc = a.ncol;
  a.cp = cat_cp.p; a.ir = cat_ir.p; a.idx_bytes = 4; a.ptr_bytes = 8; a.val = cat_val.p;
  a.val_type = DtOf<V>::value; a.on_device = 1;
  b.nrow = a.ncol; b.ncol = ncol; b.nnz = (int64_t)k * ncol; b.nzc = ncol;
  b.cp = sel_cp.p; b.ir = sel_ir.p; b.idx_bytes = 4; b.ptr_bytes = 8; b.val = nullptr;
  b.val_type = DtOf<V>::value; b.on_device = 1;
  int64_t m = 0;
  cbg_status s = dispatch_sr<V, true>(ctx, &a, &b, sr, flags, C, &m);
  HIPCHK(hipStreamSynchronize(st));   // the scratch above goes back to the pool on return
  return s;
}

}  // namespace host
}  // namespace cbg



// per-dtype entry points (defined in inst_<dtype>.hip, one translation unit each)
#define CBG_DECLARE_DT(SUF)                                                                            \
  cbg_status cbg_dispatch_##SUF(cbg_ctx*, const cbg_dcsc_view*, const cbg_dcsc_view*, cbg_semiring, uint32_t, \
                                cbg_csc_result*, int64_t*);                                            \
  cbg_status cbg_merge_##SUF(cbg_ctx*, const cbg_csc_result*, int32_t, cbg_semiring, uint32_t, cbg_csc_result*);
CBG_DECLARE_DT(f64)
CBG_DECLARE_DT(f32)
CBG_DECLARE_DT(i64)
CBG_DECLARE_DT(i32)
CBG_DECLARE_DT(b8)

// ------------------------------------------------------------------------------ duplicate summing
// A raw CSC whose columns hold rows in any order, repeated (values optional: NULL = 1) becomes a proper
// CSC -- duplicates of (row, col) summed, every column row-sorted -- as one device product
// C = I * Raw over PlusTimes<double>: each Raw nonzero gathers the single entry of one identity
// column, so the hash accumulates the duplicates in Raw's storage order (deterministic).  This is the
// SpTuples duplicate-summing constructor (SpTuples.cpp:66-115) on the device; used by the input
// builders (kron.hip) and the fused Galerkin product (galerkin.hip).
static __global__ void k_identity_csc(int64_t n, int64_t* __restrict__ cp, int32_t* __restrict__ ir) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j <= n; j += (int64_t)gridDim.x * blockDim.x) {
    cp[j] = j;
    if (j < n) ir[j] = (int32_t)j;
  }
}

inline cbg_status dedup_columns(cbg_ctx* ctx, int64_t nr, int64_t nc, int64_t nnz, const int64_t* cp,
                                const int32_t* rows, const double* val, cbg_csc_result* out) {
  hipStream_t st = ctx->stream;
  PoolBuf icp, iir;
  icp.pool = iir.pool = ctx->pool;
  HIPCHK(icp.reserve(sizeof(int64_t) * (nr + 1)));
  HIPCHK(iir.reserve(sizeof(int32_t) * (nr + 1)));
  k_identity_csc<<<(int)grid_for(nr + 1, 256, kMaxGrid), 256, 0, st>>>(nr, icp.as<int64_t>(), iir.as<int32_t>());
  HIPCHK(hipGetLastError());
  // I is A (columns trivially row-sorted, as views require); Raw is B, whose rows may come in any order
  cbg_dcsc_view a{}, b{};
  a.nrow = nr; a.ncol = nr; a.nnz = nr; a.nzc = nr;
  a.cp = icp.p; a.ir = iir.p; a.idx_bytes = 4; a.ptr_bytes = 8; a.val = nullptr; a.val_type = CBG_F64;
  a.on_device = 1;
  b.nrow = nr; b.ncol = nc; b.nnz = nnz; b.nzc = nc;
  b.cp = cp; b.ir = rows; b.idx_bytes = 4; b.ptr_bytes = 8; b.val = val; b.val_type = CBG_F64;
  b.on_device = 1;
  int64_t mult = 0;
  cbg_status s = cbg_dispatch_f64(ctx, &a, &b, CBG_SR_PLUS_TIMES, CBG_SORTED_COLS, out, &mult);
  HIPCHK(hipStreamSynchronize(st));   // the identity goes back to the pool on return
  return s;
}
