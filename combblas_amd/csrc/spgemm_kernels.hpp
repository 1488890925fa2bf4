// spgemm_kernels.hpp -- CDNA4 (gfx950) kernels of the local hash SpGEMM.
//
// Reference path (include/CombBLAS/mtSpGEMM.h): estimateFLOP 1061-1139 -> prefixsum 23-71 ->
// estimateNNZ_Hash 810-938 -> prefixsum -> numeric hash accumulate 531-642 -> integerSort -> tuples.
// Here: one pass of column statistics (flops + the row span every output column can touch),
// binning of output columns by table size, a symbolic pass (exact nnz per column), a device
// scan, and a numeric pass that emits row-sorted columns straight into the CSC result.
//
// Layout in HBM: A and B are CSC (int64 colptr[ncol+1], int32 row[nnz], V val[nnz]); C is CSC of the
// same form.  Work unit = one output column j (= one column of B).
//
// Accumulators live in LDS, one of two modes per (column, row window):
//   dense  : direct addressing over a row window of at most T rows (value slots + presence bitmap);
//            compaction is a bitmap scan, so output is sorted for free.
//   hash   : open addressing with linear probing.  Numeric uses an ORDER-PRESERVING hash
//            h(r) = ((r - lo) * T) / span so that every probe run holds keys whose home slots are in
//            the run: sorting each run locally (run-rank) yields globally sorted output.  Symbolic
//            (keys only, order irrelevant) uses a multiplicative hash.
// Every table is sized >= 2x its key count (load <= 0.5).  A numeric hash that would probe past its
// last slot (adversarial row clustering) reports the column to a fallback list that the windowed
// dense kernel processes (always correct).
//
// Parallel decomposition:
//   wave kernels  : one 64-lane wavefront per column (small columns), per-wave LDS table.
//   block kernels : one workgroup per column (medium columns), one LDS table.
//   window kernel : one workgroup per heavy column, sweeping dense row windows of 8192 rows with
//                   per-B-nonzero cursors (no re-scan, no binary search).
// Inside a column the multiplies are the union of A-column segments A(:,k), k in B(:,j).  Segments
// are processed "lane per segment" when short and "wavefront per segment" (coalesced) when long.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "semiring.hpp"

namespace cbg {
namespace {  // internal linkage: every translation unit instantiates its own kernels

constexpr int kWave = 64;
constexpr int32_t kEmpty = -1;

template <typename V>
struct DevCsc {
  int64_t nrow, ncol, nnz;
  const int64_t* cp;
  const int32_t* ir;
  const V* val;   // nullptr => pattern, all values 1/true
};

template <typename V>
__device__ __forceinline__ V load_val(const V* v, int64_t i) { return v ? v[i] : V(1); }

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }

// ---------------------------------------------------------------- wave / block scans (int32)
__device__ __forceinline__ int wave_incl_scan(int v) {
  const int l = lane_id();
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    int t = __shfl_up(v, d, kWave);
    if (l >= d) v += t;
  }
  return v;
}
__device__ __forceinline__ int64_t wave_sum64(int64_t v) {
#pragma unroll
  for (int d = kWave / 2; d > 0; d >>= 1) v += __shfl_xor(v, d, kWave);
  return v;
}

// exclusive scan over the block; `scratch` holds >= nwaves+1 ints of LDS. Contains __syncthreads.
template <int NT>
__device__ __forceinline__ int block_excl_scan(int v, int* scratch, int* total) {
  constexpr int NW = NT / kWave;
  const int w = threadIdx.x / kWave, l = lane_id();
  int inc = wave_incl_scan(v);
  if (l == kWave - 1) scratch[w] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    int run = 0;
    for (int i = 0; i < NW; ++i) { int t = scratch[i]; scratch[i] = run; run += t; }
    scratch[NW] = run;
  }
  __syncthreads();
  int ex = scratch[w] + inc - v;
  *total = scratch[NW];
  __syncthreads();
  return ex;
}

// ============================================================================ 1. column statistics
// flop[j] = sum_{k in B(:,j)} nnz(A(:,k))   (estimateFLOP, mtSpGEMM.h:1117-1135)
// span[j] = [min, max] row index any of those A columns holds (A columns are row-sorted).
// 16 lanes per column.
template <typename VB>
__global__ void __launch_bounds__(256) k_col_stats(int64_t ncol, const int64_t* __restrict__ Acp,
                                                   const int32_t* __restrict__ Air,
                                                   const int64_t* __restrict__ Bcp,
                                                   const int32_t* __restrict__ Bir,
                                                   int64_t* __restrict__ flop, int2* __restrict__ span,
                                                   unsigned long long* __restrict__ total) {
  const int64_t gid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t j = gid >> 4;
  const int sub = threadIdx.x & 15;
  int64_t f = 0;
  int lo = INT32_MAX, hi = -1;
  if (j < ncol) {
    const int64_t e = Bcp[j + 1];
    for (int64_t p = Bcp[j] + sub; p < e; p += 16) {
      const int32_t k = Bir[p];
      const int64_t a0 = Acp[k], a1 = Acp[k + 1];
      if (a1 > a0) {
        f += a1 - a0;
        lo = min(lo, Air[a0]);
        hi = max(hi, Air[a1 - 1]);
      }
    }
  }
#pragma unroll
  for (int d = 8; d > 0; d >>= 1) {
    f += __shfl_xor(f, d, 16);
    lo = min(lo, __shfl_xor(lo, d, 16));
    hi = max(hi, __shfl_xor(hi, d, 16));
  }
  if (sub == 0 && j < ncol) {
    flop[j] = f;
    span[j] = make_int2(lo, hi);
  }
  // block-level total of multiplies
  __shared__ unsigned long long s_tot;
  if (threadIdx.x == 0) s_tot = 0;
  __syncthreads();
  int64_t wf = (sub == 0) ? f : 0;
  wf = wave_sum64(wf);
  if (lane_id() == 0 && wf) atomicAdd(&s_tot, (unsigned long long)wf);
  __syncthreads();
  if (threadIdx.x == 0 && s_tot) atomicAdd(total, s_tot);
}

// ============================================================================ 2. binning
// Class ids (shared by symbolic and numeric binning, different size meaning):
//   0              : empty column (nothing to do)
//   1..NWC         : wave classes, table T = 64 << (c-1)
//   NWC+1..NWC+NBC : block classes, table T = (64 << NWC) << (c-1-NWC)
//   NWC+NBC+1      : windowed (heavy) class
struct BinParams {
  int nwave, nblock;     // number of wave / block classes
  int64_t wave_min_T;    // 64
  int sym;               // 1: symbolic (need = min(2*flop, ceil(span/32)) words); 0: numeric (need = min(2*nnz, span) slots)
};

__device__ __forceinline__ int class_of(int64_t need, const BinParams& bp) {
  if (need <= 0) return 0;
  int64_t T = bp.wave_min_T;
  const int ntot = bp.nwave + bp.nblock;
  for (int c = 1; c <= ntot; ++c, T <<= 1)
    if (need <= T) return c;
  return ntot + 1;
}

__device__ __forceinline__ int64_t need_of(int64_t cnt, int2 sp, int sym) {
  if (cnt <= 0 || sp.y < sp.x) return 0;
  const int64_t span = (int64_t)sp.y - sp.x + 1;
  if (sym) return min(2 * cnt, (span + 31) / 32);
  return min(2 * cnt, span);
}

// pass 0: histogram; pass 1: scatter into class-contiguous list using device cursors
__global__ void __launch_bounds__(256) k_bin(int64_t ncol, const int64_t* __restrict__ cnt,
                                             const int2* __restrict__ span, BinParams bp, int pass,
                                             unsigned long long* __restrict__ hist,
                                             unsigned long long* __restrict__ cursor,
                                             int32_t* __restrict__ list) {
  __shared__ unsigned int s_h[32];
  __shared__ unsigned long long s_base[32];
  const int ncls = bp.nwave + bp.nblock + 2;
  if (threadIdx.x < 32) s_h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  int c = -1;
  unsigned int rank = 0;
  if (j < ncol) {
    c = class_of(need_of(cnt[j], span[j], bp.sym), bp);
    rank = atomicAdd(&s_h[c], 1u);
  }
  __syncthreads();
  if (pass == 0) {
    if (threadIdx.x < ncls && s_h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], (unsigned long long)s_h[threadIdx.x]);
    return;
  }
  if (threadIdx.x < ncls) s_base[threadIdx.x] = s_h[threadIdx.x] ? atomicAdd(&cursor[threadIdx.x], (unsigned long long)s_h[threadIdx.x]) : 0;
  __syncthreads();
  if (c >= 0) list[s_base[c] + rank] = (int32_t)j;
}

// ============================================================================ accumulation helpers
// Table views in LDS
template <typename Acc>
struct Table {
  int32_t* keys;   // hash: keys[Tcap]; dense: presence bitmap (T/32 words)
  Acc* vals;       // T (dense) or Tcap (hash) slots
  int32_t T;       // home range (hash) / window rows (dense)
  int32_t Tcap;    // hash: T + tail pad
};

// order-preserving hash: home = ((r - lo) * mult) >> 32, mult = floor(2^32 * T / span)
__device__ __forceinline__ uint32_t mono_home(int32_t r, int32_t lo, uint32_t mult) {
  return __umulhi((uint32_t)(r - lo), mult);
}

// numeric insert into an order-preserving hash table; returns false on overflow.
template <class SRT>
__device__ __forceinline__ bool hash_insert_num(Table<typename SRT::Acc>& t, int32_t r, uint32_t home,
                                                typename SRT::Acc x, int* adderr) {
  int32_t s = (int32_t)home;
  while (s < t.Tcap) {
    int32_t cur = t.keys[s];
    if (cur == kEmpty) cur = atomicCAS(&t.keys[s], kEmpty, r);
    if (cur == kEmpty || cur == r) {
      if (SRT::kAddIsError && cur == r) *adderr = 1;
      SRT::acc(&t.vals[s], x);
      return true;
    }
    ++s;
  }
  return false;
}

__device__ __forceinline__ uint32_t sym_home(int32_t r, int32_t logT) {
  return ((uint32_t)r * 2654435761u) >> (32 - logT);
}
// symbolic insert (keys only, wrap-around probing); returns 1 if the key is new
__device__ __forceinline__ int hash_insert_sym(int32_t* keys, int32_t r, int32_t logT) {
  const uint32_t mask = (1u << logT) - 1;
  uint32_t s = sym_home(r, logT);
  for (;;) {
    int32_t cur = keys[s];
    if (cur == r) return 0;
    if (cur == kEmpty) {
      cur = atomicCAS(&keys[s], kEmpty, r);
      if (cur == kEmpty) return 1;
      if (cur == r) return 0;
    }
    s = (s + 1) & mask;
  }
}

// ============================================================================ segment expansion
// Visit every multiply (q in A(:,k), b in B(:,j)) of column j with a group of NT lanes
// (NT = 64 for a wavefront, or the block size).  Short segments (< kLong entries): one lane walks
// the segment.  Long segments: a whole wavefront walks it in coalesced 64-entry strides.
// F(q, b) is called once per multiply.  The caller provides LDS for the long-segment queue.
constexpr int kLong = 64;

template <int NT, bool WAVE_ONLY, typename F>
__device__ __forceinline__ void for_each_multiply(int64_t bs, int64_t be, const int64_t* __restrict__ Acp,
                                                  const int32_t* __restrict__ Bir, int32_t* lq, int* lq_n,
                                                  F&& f) {
  const int tid = WAVE_ONLY ? lane_id() : (int)threadIdx.x;
  for (int64_t base = bs; base < be; base += NT) {
    const int64_t b = base + tid;
    int64_t a0 = 0, a1 = 0;
    if (b < be) {
      const int32_t k = Bir[b];
      a0 = Acp[k];
      a1 = Acp[k + 1];
    }
    const bool islong = (a1 - a0) >= kLong;
    if (!islong) {
      for (int64_t q = a0; q < a1; ++q) f(q, b);
    }
    // long segments: queue them (LDS), then each wavefront takes queue entries round-robin
    if constexpr (WAVE_ONLY) {
      const unsigned long long m = __ballot(islong);
      const int pos = __popcll(m & ((1ull << lane_id()) - 1));
      if (islong) lq[pos] = tid;   // store lane index; segment recomputed below
      wave_sync();
      const int nl = __popcll(m);
      for (int i = 0; i < nl; ++i) {
        const int src = lq[i];
        const int64_t sb = base + src;
        const int64_t s0 = __shfl(a0, src, kWave), s1 = __shfl(a1, src, kWave);
        for (int64_t q = s0 + lane_id(); q < s1; q += kWave) f(q, sb);
      }
      wave_sync();
    } else {
      if (threadIdx.x == 0) *lq_n = 0;
      __syncthreads();
      if (islong) lq[atomicAdd(lq_n, 1)] = tid;
      __syncthreads();
      const int nl = *lq_n;
      const int w = threadIdx.x / kWave;
      constexpr int NW = NT / kWave;
      for (int i = w; i < nl; i += NW) {
        const int64_t sb = base + lq[i];
        const int32_t k = Bir[sb];
        const int64_t s0 = Acp[k], s1 = Acp[k + 1];
        for (int64_t q = s0 + lane_id(); q < s1; q += kWave) f(q, sb);
      }
      __syncthreads();
    }
  }
}

// ============================================================================ 3. symbolic
// Exact nnz of C(:,j) (estimateNNZ_Hash, mtSpGEMM.h:866-933).  Mode per column: presence bitmap over
// the column's row span when it fits the class table, else a keys-only hash with T >= 2*flop.
template <int LOGT>
struct SymWaveCfg { static constexpr int T = 1 << LOGT; };

// wave kernel: 4 wavefronts per 256-thread block, one column per wavefront at a time
template <int LOGT>
__global__ void __launch_bounds__(256) k_sym_wave(const int32_t* __restrict__ list, int64_t count,
                                                  const int64_t* __restrict__ Acp, const int32_t* __restrict__ Air,
                                                  const int64_t* __restrict__ Bcp, const int32_t* __restrict__ Bir,
                                                  const int2* __restrict__ span, int64_t* __restrict__ nnz) {
  constexpr int T = 1 << LOGT;
  __shared__ int32_t s_tab[4][T];
  __shared__ int32_t s_lq[4][kWave];
  const int w = threadIdx.x / kWave, l = lane_id();
  int32_t* tab = s_tab[w];
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  for (int64_t i = blockIdx.x * 4 + w; i < count; i += nwaves) {
    const int32_t j = list[i];
    const int2 sp = span[j];
    const int64_t spn = (int64_t)sp.y - sp.x + 1;
    const bool bitmap = spn <= 32LL * T;
    for (int s = l; s < T; s += kWave) tab[s] = bitmap ? 0 : kEmpty;
    wave_sync();
    int cnt = 0;
    for_each_multiply<kWave, true>(Bcp[j], Bcp[j + 1], Acp, Bir, s_lq[w], nullptr, [&](int64_t q, int64_t) {
      const int32_t r = Air[q];
      if (bitmap) {
        const int32_t o = r - sp.x;
        const uint32_t bit = 1u << (o & 31);
        if (!(tab[o >> 5] & bit)) cnt += (atomicOr((uint32_t*)&tab[o >> 5], bit) & bit) ? 0 : 1;
      } else {
        cnt += hash_insert_sym(tab, r, LOGT);
      }
    });
    int64_t tot = wave_sum64(cnt);
    if (l == 0) nnz[j] = tot;
    wave_sync();
  }
}

// block kernel: one column per workgroup
template <int LOGT, int NT>
__global__ void __launch_bounds__(NT) k_sym_block(const int32_t* __restrict__ list, int64_t count,
                                                  const int64_t* __restrict__ Acp, const int32_t* __restrict__ Air,
                                                  const int64_t* __restrict__ Bcp, const int32_t* __restrict__ Bir,
                                                  const int2* __restrict__ span, int64_t* __restrict__ nnz) {
  constexpr int T = 1 << LOGT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int32_t* tab = (int32_t*)smem;
  int32_t* lq = tab + T;          // NT
  int* misc = lq + NT;            // [0] queue count, [1] total
  for (int64_t i = blockIdx.x; i < count; i += gridDim.x) {
    const int32_t j = list[i];
    const int2 sp = span[j];
    const int64_t spn = (int64_t)sp.y - sp.x + 1;
    const bool bitmap = spn <= 32LL * T;
    for (int s = threadIdx.x; s < T; s += NT) tab[s] = bitmap ? 0 : kEmpty;
    if (threadIdx.x == 0) misc[1] = 0;
    __syncthreads();
    int cnt = 0;
    for_each_multiply<NT, false>(Bcp[j], Bcp[j + 1], Acp, Bir, lq, &misc[0], [&](int64_t q, int64_t) {
      const int32_t r = Air[q];
      if (bitmap) {
        const int32_t o = r - sp.x;
        const uint32_t bit = 1u << (o & 31);
        if (!(tab[o >> 5] & bit)) cnt += (atomicOr((uint32_t*)&tab[o >> 5], bit) & bit) ? 0 : 1;
      } else {
        cnt += hash_insert_sym(tab, r, LOGT);
      }
    });
    int64_t wc = wave_sum64(cnt);
    if (lane_id() == 0 && wc) atomicAdd(&misc[1], (int)wc);
    __syncthreads();
    if (threadIdx.x == 0) nnz[j] = misc[1];
    __syncthreads();
  }
}

// ============================================================================ 4. scan
// exclusive scan of int64 counts into colptr[n+1]; 3 kernels, tile = 1024 elements
constexpr int kScanTile = 1024;
__global__ void __launch_bounds__(256) k_scan_tiles(int64_t n, const int64_t* __restrict__ in,
                                                    int64_t* __restrict__ tile_sum) {
  __shared__ int64_t s[4];
  const int64_t base = blockIdx.x * (int64_t)kScanTile;
  int64_t v = 0;
  for (int i = threadIdx.x; i < kScanTile; i += 256)
    if (base + i < n) v += in[base + i];
  v = wave_sum64(v);
  if (lane_id() == 0) s[threadIdx.x / kWave] = v;
  __syncthreads();
  if (threadIdx.x == 0) tile_sum[blockIdx.x] = s[0] + s[1] + s[2] + s[3];
}
__global__ void __launch_bounds__(1024) k_scan_sums(int64_t ntiles, int64_t* __restrict__ tile_sum,
                                                    int64_t* __restrict__ total) {
  __shared__ int64_t s[17];
  __shared__ int64_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int64_t base = 0; base < ntiles; base += 1024) {
    const int64_t i = base + threadIdx.x;
    int64_t v = i < ntiles ? tile_sum[i] : 0;
    int64_t inc = v;
    const int l = lane_id();
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
      int64_t t = __shfl_up(inc, d, kWave);
      if (l >= d) inc += t;
    }
    const int w = threadIdx.x / kWave;
    if (l == kWave - 1) s[w] = inc;
    __syncthreads();
    if (threadIdx.x == 0) {
      int64_t run = 0;
      for (int q = 0; q < 16; ++q) { int64_t t = s[q]; s[q] = run; run += t; }
      s[16] = run;
    }
    __syncthreads();
    if (i < ntiles) tile_sum[i] = carry + s[w] + inc - v;
    __syncthreads();
    if (threadIdx.x == 0) carry += s[16];
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = carry;
}
__global__ void __launch_bounds__(256) k_scan_apply(int64_t n, const int64_t* __restrict__ in,
                                                    const int64_t* __restrict__ tile_off,
                                                    int64_t* __restrict__ out) {
  __shared__ int64_t s[5];
  const int64_t base = blockIdx.x * (int64_t)kScanTile;
  // each thread owns 4 consecutive elements
  int64_t v[4], t = 0;
  for (int e = 0; e < 4; ++e) {
    const int64_t i = base + threadIdx.x * 4 + e;
    v[e] = i < n ? in[i] : 0;
    t += v[e];
  }
  int64_t inc = t;
  const int l = lane_id();
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    int64_t u = __shfl_up(inc, d, kWave);
    if (l >= d) inc += u;
  }
  const int w = threadIdx.x / kWave;
  if (l == kWave - 1) s[w] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t run = 0;
    for (int q = 0; q < 4; ++q) { int64_t u = s[q]; s[q] = run; run += u; }
  }
  __syncthreads();
  int64_t run = tile_off[blockIdx.x] + s[w] + inc - t;
  if (blockIdx.x == 0 && threadIdx.x == 0) out[0] = 0;
  for (int e = 0; e < 4; ++e) {
    const int64_t i = base + threadIdx.x * 4 + e;
    run += v[e];
    if (i < n) out[i + 1] = run;
  }
}

// ============================================================================ 5. numeric
// Output: C.row / C.val at colptr[j] .. colptr[j+1], rows ascending.
template <typename V>
struct NumOut {
  const int64_t* colptr;
  int32_t* row;
  V* val;
  int* adderr;            // BoolCopy add() attempted
  int* overflow_n;        // fallback list length
  int32_t* overflow_list; // columns whose order-preserving hash overflowed
};

// Compaction of an order-preserving hash table of Tcap slots by `NT` lanes (tid in [0,NT)).
// out position of an occupied slot s = (#occupied before its run start) + (#keys in its run smaller).
template <int NT, class SRT, typename V>
__device__ __forceinline__ void compact_hash_runs(const int32_t* keys, const typename SRT::Acc* vals, int Tcap,
                                                  int tid, int occ_before_chunk, int c0, int c1, int64_t outbase,
                                                  const V* aval, const V* bval, int32_t* orow, V* oval) {
  int occ = occ_before_chunk;
  for (int s = c0; s < c1; ++s) {
    const int32_t key = keys[s];
    if (key == kEmpty) continue;
    int rs = s;
    while (rs > 0 && keys[rs - 1] != kEmpty) --rs;
    int smaller = 0;
    for (int t = rs; t < Tcap; ++t) {
      const int32_t kt = keys[t];
      if (kt == kEmpty) break;
      smaller += (kt < key);
    }
    const int64_t o = outbase + (occ - (s - rs)) + smaller;
    orow[o] = key;
    oval[o] = SRT::out(vals[s], aval, bval);
    ++occ;
  }
}

// ---- wave numeric: one column per wavefront, table T slots (+kTail) per wave
constexpr int kTail = 64;

template <class SRT, typename V, int LOGT>
__global__ void __launch_bounds__(256) k_num_wave(const int32_t* __restrict__ list, int64_t count,
                                                  DevCsc<V> A, DevCsc<V> B, const int2* __restrict__ span,
                                                  NumOut<V> out) {
  using Acc = typename SRT::Acc;
  constexpr int T = 1 << LOGT;
  constexpr int TC = T + kTail;
  __shared__ int32_t s_keys[4][TC];
  __shared__ Acc s_vals[4][TC];
  __shared__ int32_t s_lq[4][kWave];
  const int w = threadIdx.x / kWave, l = lane_id();
  Table<Acc> t{s_keys[w], s_vals[w], T, TC};
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  for (int64_t i = blockIdx.x * 4 + w; i < count; i += nwaves) {
    const int32_t j = list[i];
    const int2 sp = span[j];
    const int64_t spn = (int64_t)sp.y - sp.x + 1;
    const bool dense = spn <= T;
    const uint32_t mult = dense ? 0u : (uint32_t)(((uint64_t)T << 32) / (uint64_t)spn);
    for (int s = l; s < TC; s += kWave) { t.keys[s] = dense ? 0 : kEmpty; t.vals[s] = SRT::identity(); }
    wave_sync();
    int ovf = 0, aerr = 0;
    for_each_multiply<kWave, true>(B.cp[j], B.cp[j + 1], A.cp, B.ir, s_lq[w], nullptr, [&](int64_t q, int64_t b) {
      const int32_t r = A.ir[q];
      const Acc x = SRT::mul(load_val(A.val, q), load_val(B.val, b), q, b);
      if (dense) {
        const int32_t o = r - sp.x;
        const uint32_t bit = 1u << (o & 31);
        const uint32_t old = atomicOr((uint32_t*)&t.keys[o >> 5], bit);
        if (SRT::kAddIsError && (old & bit)) aerr = 1;
        SRT::acc(&t.vals[o], x);
      } else {
        if (!hash_insert_num<SRT>(t, r, mono_home(r, sp.x, mult), x, &aerr)) ovf = 1;
      }
    });
    wave_sync();
    const bool wov = __any(ovf);
    if (__any(aerr) && l == 0) atomicOr(out.adderr, 1);
    const int64_t ob = out.colptr[j];
    if (wov) {
      if (l == 0) out.overflow_list[atomicAdd(out.overflow_n, 1)] = j;
    } else if (dense) {
      // bitmap words: T/32 <= 16 for T <= 512 -> lanes 0..T/32-1
      constexpr int NWORD = T / 32;
      uint32_t wd = (l < NWORD) ? (uint32_t)t.keys[l] : 0u;
      const int pc = __popc(wd);
      const int ex = wave_incl_scan(pc) - pc;
      int o = ex;
      while (wd) {
        const int bpos = __ffs(wd) - 1;
        wd &= wd - 1;
        const int rr = l * 32 + bpos;
        out.row[ob + o] = sp.x + rr;
        out.val[ob + o] = SRT::out(t.vals[rr], A.val, B.val);
        ++o;
      }
    } else {
      // chunk of TC/64 slots per lane (TC multiple of 64)
      constexpr int CH = TC / kWave;
      const int c0 = l * CH, c1 = c0 + CH;
      int occ = 0;
      for (int s = c0; s < c1; ++s) occ += (t.keys[s] != kEmpty);
      const int ex = wave_incl_scan(occ) - occ;
      compact_hash_runs<kWave, SRT, V>(t.keys, t.vals, TC, l, ex, c0, c1, ob, A.val, B.val, out.row, out.val);
    }
    wave_sync();
  }
}

// ---- block numeric: one column per workgroup; LDS = TC*(4+sizeof(Acc)) + small
template <class SRT, typename V, int LOGT, int NT>
__global__ void __launch_bounds__(NT) k_num_block(const int32_t* __restrict__ list, int64_t count,
                                                  DevCsc<V> A, DevCsc<V> B, const int2* __restrict__ span,
                                                  NumOut<V> out) {
  using Acc = typename SRT::Acc;
  constexpr int T = 1 << LOGT;
  constexpr int TC = T + NT;      // tail = one slot per thread keeps chunks uniform
  extern __shared__ __attribute__((aligned(16))) char smem[];
  Acc* vals = (Acc*)smem;
  int32_t* keys = (int32_t*)(vals + TC);
  int32_t* lq = keys + TC;        // NT
  int* misc = lq + NT;            // [0] lq count, [1] overflow, [2] adderr, [3..] scan scratch
  Table<Acc> t{keys, vals, T, TC};
  for (int64_t i = blockIdx.x; i < count; i += gridDim.x) {
    const int32_t j = list[i];
    const int2 sp = span[j];
    const int64_t spn = (int64_t)sp.y - sp.x + 1;
    const bool dense = spn <= T;
    const uint32_t mult = dense ? 0u : (uint32_t)(((uint64_t)T << 32) / (uint64_t)spn);
    for (int s = threadIdx.x; s < TC; s += NT) { keys[s] = dense ? 0 : kEmpty; vals[s] = SRT::identity(); }
    if (threadIdx.x == 0) { misc[1] = 0; misc[2] = 0; }
    __syncthreads();
    int ovf = 0, aerr = 0;
    for_each_multiply<NT, false>(B.cp[j], B.cp[j + 1], A.cp, B.ir, lq, &misc[0], [&](int64_t q, int64_t b) {
      const int32_t r = A.ir[q];
      const Acc x = SRT::mul(load_val(A.val, q), load_val(B.val, b), q, b);
      if (dense) {
        const int32_t o = r - sp.x;
        const uint32_t bit = 1u << (o & 31);
        const uint32_t old = atomicOr((uint32_t*)&keys[o >> 5], bit);
        if (SRT::kAddIsError && (old & bit)) aerr = 1;
        SRT::acc(&vals[o], x);
      } else {
        if (!hash_insert_num<SRT>(t, r, mono_home(r, sp.x, mult), x, &aerr)) ovf = 1;
      }
    });
    if (ovf) misc[1] = 1;
    if (aerr) misc[2] = 1;
    __syncthreads();
    const int64_t ob = out.colptr[j];
    if (misc[1]) {
      if (threadIdx.x == 0) out.overflow_list[atomicAdd(out.overflow_n, 1)] = j;
    } else if (dense) {
      // presence bitmap: T/32 words; word w owned by thread w (T/32 <= NT for T <= 32*NT)
      const int NWORD = T / 32;
      uint32_t wd = (threadIdx.x < NWORD) ? (uint32_t)keys[threadIdx.x] : 0u;
      int tot;
      int o = block_excl_scan<NT>(__popc(wd), misc + 3, &tot);
      while (wd) {
        const int bpos = __ffs(wd) - 1;
        wd &= wd - 1;
        const int rr = threadIdx.x * 32 + bpos;
        out.row[ob + o] = sp.x + rr;
        out.val[ob + o] = SRT::out(vals[rr], A.val, B.val);
        ++o;
      }
    } else {
      constexpr int CH = TC / NT;
      const int c0 = threadIdx.x * CH, c1 = c0 + CH;
      int occ = 0;
      for (int s = c0; s < c1; ++s) occ += (keys[s] != kEmpty);
      int tot;
      const int ex = block_excl_scan<NT>(occ, misc + 3, &tot);
      compact_hash_runs<NT, SRT, V>(keys, vals, TC, threadIdx.x, ex, c0, c1, ob, A.val, B.val, out.row, out.val);
    }
    if (threadIdx.x == 0 && misc[2]) atomicOr(out.adderr, 1);
    __syncthreads();
  }
}

// ============================================================================ 6. windowed (heavy)
// One workgroup per column, sweeping row windows [r0, r0+W) over the column's span.  Every B nonzero
// b of the column owns a cursor into A(:,k) (cur[b], absolute index) and caches the row at the
// cursor (nxt[b]); a window only touches segments whose cached row is inside it.
// MODE 0 = symbolic (presence bitmap, count only), MODE 1 = numeric (dense value window + bitmap).
constexpr int kWinRows = 8192;         // numeric dense window (64 KB of f64 values)
constexpr int kSymWinRows = 1 << 20;   // symbolic bitmap window (128 KB)

template <int MODE, class SRT, typename V, int NT, int W>
__global__ void __launch_bounds__(NT) k_window(const int32_t* __restrict__ list, const int* __restrict__ count_dev,
                                               int64_t count_host, DevCsc<V> A, DevCsc<V> B,
                                               const int2* __restrict__ span, int64_t* __restrict__ cur,
                                               int32_t* __restrict__ nxt, int64_t* __restrict__ nnz, NumOut<V> out) {
  using Acc = typename SRT::Acc;
  constexpr int NWORD = W / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  Acc* vals = (Acc*)smem;                                    // W (MODE 1) or 0
  uint32_t* bits = (uint32_t*)(vals + (MODE == 1 ? W : 0));  // NWORD
  int32_t* lq = (int32_t*)(bits + NWORD);                    // NT (queue of long segments)
  int* misc = lq + NT;                                       // [0] lq n, [1] count, [2] adderr, [3..] scan
  const int64_t count = count_dev ? (int64_t)*count_dev : count_host;
  for (int64_t i = blockIdx.x; i < count; i += gridDim.x) {
    const int32_t j = list[i];
    const int2 sp = span[j];
    const int64_t bs = B.cp[j], be = B.cp[j + 1];
    // init cursors
    for (int64_t b = bs + threadIdx.x; b < be; b += NT) {
      const int32_t k = B.ir[b];
      const int64_t a0 = A.cp[k], a1 = A.cp[k + 1];
      cur[b] = a0;
      nxt[b] = a0 < a1 ? A.ir[a0] : INT32_MAX;
    }
    if (threadIdx.x == 0) misc[2] = 0;
    __syncthreads();
    int64_t outpos = (MODE == 1) ? out.colptr[j] : 0;
    int64_t total = 0;
    int aerr = 0;
    for (int64_t r0 = sp.x; r0 <= sp.y; r0 += W) {
      const int32_t r1 = (int32_t)min<int64_t>(r0 + W, (int64_t)sp.y + 1);
      for (int s = threadIdx.x; s < NWORD; s += NT) bits[s] = 0u;
      if constexpr (MODE == 1)
        for (int s = threadIdx.x; s < W; s += NT) vals[s] = SRT::identity();
      __syncthreads();
      // visit segments with work in this window
      for (int64_t base = bs; base < be; base += NT) {
        const int64_t b = base + threadIdx.x;
        int64_t q = 0, qe = 0;
        bool act = false;
        if (b < be) {
          const int32_t r = nxt[b];
          if (r < r1) {
            act = true;
            q = cur[b];
            qe = A.cp[B.ir[b] + 1];
          }
        }
        // long-in-window test: a segment with >= 64 entries left is handed to a wavefront
        const bool islong = act && (qe - q) >= kLong && A.ir[q + kLong - 1] < r1;
        if (act && !islong) {
          const V bv = load_val(B.val, b);
          int32_t r = nxt[b];
          while (true) {
            const int32_t o = r - (int32_t)r0;
            const uint32_t bit = 1u << (o & 31);
            if constexpr (MODE == 0) {
              if (!(bits[o >> 5] & bit)) atomicOr(&bits[o >> 5], bit);
            } else {
              const uint32_t old = atomicOr(&bits[o >> 5], bit);
              if (SRT::kAddIsError && (old & bit)) aerr = 1;
              SRT::acc(&vals[o], SRT::mul(load_val(A.val, q), bv, q, b));
            }
            ++q;
            if (q >= qe) { r = INT32_MAX; break; }
            r = A.ir[q];
            if (r >= r1) break;
          }
          cur[b] = q;
          nxt[b] = r;
        }
        if (threadIdx.x == 0) misc[0] = 0;
        __syncthreads();
        if (islong) lq[atomicAdd(&misc[0], 1)] = threadIdx.x;
        __syncthreads();
        const int nl = misc[0];
        for (int e = threadIdx.x / kWave; e < nl; e += NT / kWave) {
          const int64_t sb = base + lq[e];
          int64_t sq = cur[sb];
          const int64_t sqe = A.cp[B.ir[sb] + 1];
          const V bv = load_val(B.val, sb);
          int32_t rn = INT32_MAX;
          while (true) {
            const int64_t qq = sq + lane_id();
            const int32_t r = qq < sqe ? A.ir[qq] : INT32_MAX;
            const bool in = r < r1;
            if (in) {
              const int32_t o = r - (int32_t)r0;
              const uint32_t bit = 1u << (o & 31);
              if constexpr (MODE == 0) {
                atomicOr(&bits[o >> 5], bit);
              } else {
                const uint32_t old = atomicOr(&bits[o >> 5], bit);
                if (SRT::kAddIsError && (old & bit)) aerr = 1;
                SRT::acc(&vals[o], SRT::mul(load_val(A.val, qq), bv, qq, sb));
              }
            }
            const unsigned long long m = __ballot(in);
            const int nin = __popcll(m);
            sq += nin;
            if (nin < kWave) {
              // first lane not in window holds the next row (or INT32_MAX past the end)
              const int fl = __ffsll((long long)~m) - 1;
              rn = __shfl(r, fl, kWave);
              break;
            }
          }
          if (lane_id() == 0) { cur[sb] = sq; nxt[sb] = rn; }
        }
        __syncthreads();
      }
      // compaction of this window
      int wcnt = 0;
      for (int s = threadIdx.x; s < NWORD; s += NT) wcnt += __popc(bits[s]);
      int tot;
      if constexpr (MODE == 0) {
        int64_t ws = wave_sum64(wcnt);
        if (threadIdx.x == 0) misc[1] = 0;
        __syncthreads();
        if (lane_id() == 0 && ws) atomicAdd(&misc[1], (int)ws);
        __syncthreads();
        total += misc[1];
        __syncthreads();
      } else {
        // thread owns words [tid*PW, tid*PW+PW), PW = NWORD/NT
        constexpr int PW = NWORD / NT;
        static_assert(NWORD % NT == 0, "window words must split evenly");
        int c = 0;
        for (int s = 0; s < PW; ++s) c += __popc(bits[threadIdx.x * PW + s]);
        int o = block_excl_scan<NT>(c, misc + 3, &tot);
        for (int s = 0; s < PW; ++s) {
          uint32_t wd = bits[threadIdx.x * PW + s];
          while (wd) {
            const int bpos = __ffs(wd) - 1;
            wd &= wd - 1;
            const int rr = (threadIdx.x * PW + s) * 32 + bpos;
            out.row[outpos + o] = (int32_t)r0 + rr;
            out.val[outpos + o] = SRT::out(vals[rr], A.val, B.val);
            ++o;
          }
        }
        outpos += tot;
        __syncthreads();
      }
    }
    if (MODE == 0 && threadIdx.x == 0) nnz[j] = total;
    if (MODE == 1) {
      if (aerr) misc[2] = 1;
      __syncthreads();
      if (threadIdx.x == 0 && misc[2]) atomicOr(out.adderr, 1);
    }
    __syncthreads();
  }
}

// ============================================================================ misc device utilities
__global__ void k_widen_idx(int64_t n, const int64_t* __restrict__ in, int32_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (int32_t)in[i];
}
__global__ void k_i32_to_i64(int64_t n, const int32_t* __restrict__ in, int64_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = in[i];
}
// DCSC (cp[nzc+1], jc[nzc]) -> dense colptr[ncol+1]: colptr[c] = cp[first jc >= c]
__global__ void k_dcsc_to_csc(int64_t ncol, int64_t nzc, const int64_t* __restrict__ cp,
                              const int64_t* __restrict__ jc, int64_t* __restrict__ colptr) {
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c <= ncol; c += (int64_t)gridDim.x * blockDim.x) {
    int64_t lo = 0, hi = nzc;   // first index with jc >= c
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (jc[mid] < c) lo = mid + 1; else hi = mid;
    }
    colptr[c] = cp[lo];
  }
}

}  // namespace
}  // namespace cbg
