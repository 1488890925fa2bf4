// spgemm_kernels.hpp -- CDNA4 (gfx950) kernels of the local hash SpGEMM.
//
// Reference path (include/CombBLAS/mtSpGEMM.h): estimateFLOP 1061-1139 -> prefixsum 23-71 ->
// estimateNNZ_Hash 810-938 -> prefixsum -> numeric hash accumulate 531-642 -> integerSort -> tuples.
// Here: one pass of column statistics (flops + the row span every output column can touch),
// binning of output columns by table size, a symbolic pass (exact nnz per column), a device
// scan, and a numeric pass that emits row-sorted columns straight into the CSC result.
//
// Layout in HBM: A and B are CSC (int64 colptr[ncol+1], int32 row[nnz], V val[nnz]); C is CSC of the
// same form.  Work item = one output column j (= one column of B), or, for heavy columns, one UNIT:
// a row range of column j aligned to SUBW-row subwindows, holding at most kUnitCap outputs.
//
// Accumulators live in LDS, one of two modes per work item:
//   dense  : direct addressing over a row range of at most T rows (value slots + presence bitmap);
//            compaction is a bitmap scan, so output is sorted for free.
//   hash   : open addressing with linear probing.  Numeric uses an ORDER-PRESERVING hash
//            h(r) = ((r - lo) * T) / span so that every probe run holds keys whose home slots are in
//            the run: sorting each run locally (run-rank) yields globally sorted output.  Symbolic
//            (keys only, order irrelevant) uses a multiplicative hash.
// Every table is sized >= 2x its key count (load <= 0.5).  A numeric hash that would probe past its
// last slot (adversarial row clustering) hands the work item to a fallback that is always correct.
//
// Heavy columns (nnz > kHeavy): the symbolic pass records the column's nnz per SUBW-row subwindow;
// units are formed from consecutive subwindows (exact counts -> exact output offsets), and the A
// segment of a unit is found without search through a split table (relative offsets of every
// subwindow boundary inside each long A column).  Units are independent, so a column with 250k
// outputs spreads over ~60 workgroups instead of one.
//
// Inside a work item the multiplies are the union of A-column segments A(:,k), k in B(:,j); they are
// flattened and dealt to lanes evenly (for_each_multiply), so power-law segment lengths cost no
// imbalance and every lane keeps kUnroll independent gathers in flight.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "semiring.hpp"

namespace cbg {
namespace {  // internal linkage: every translation unit instantiates its own kernels

constexpr int kWave = 64;
constexpr int32_t kEmpty = -1;
constexpr int kLong = 64;          // k_window: segment length handed to a whole wavefront
#ifndef CBG_UNROLL_NUM
#define CBG_UNROLL_NUM 2
#endif
#ifndef CBG_UNROLL_SYM
#define CBG_UNROLL_SYM 2
#endif
#ifndef CBG_GROUP_SYM
#define CBG_GROUP_SYM 4
#endif
#ifndef CBG_GROUP_NUM
#define CBG_GROUP_NUM 2
#endif
constexpr int kUnroll = CBG_UNROLL_NUM;       // groups of G multiplies in flight per lane (numeric)
constexpr int kUnrollSym = CBG_UNROLL_SYM;    // same, symbolic (4-byte items)
#ifndef CBG_UNROLL_HEAVY
#define CBG_UNROLL_HEAVY 1
#endif
#ifndef CBG_GROUP_HEAVY
#define CBG_GROUP_HEAVY 4
#endif
constexpr int kUnrollHeavy = CBG_UNROLL_HEAVY;    // same, k_num_heavy
constexpr int kGroupSym = CBG_GROUP_SYM;  // consecutive A entries per lane group (one segment search each), symbolic
constexpr int kGroupNum = CBG_GROUP_NUM;  // same, numeric
constexpr int kGroupHeavy = CBG_GROUP_HEAVY;     // same, k_num_heavy
#ifndef CBG_HEAVY_MIN
#define CBG_HEAVY_MIN 4096
#endif
constexpr int64_t kHeavy = CBG_HEAVY_MIN;   // nnz(C(:,j)) above which a column is split into units
// k_num_heavy geometry: table 2^CBG_HEAVY_LOGT slots, CBG_HEAVY_NT threads (LDS decides WGs per CU)
#ifndef CBG_HEAVY_LOGT
#define CBG_HEAVY_LOGT 13
#endif
#ifndef CBG_HEAVY_NT
#define CBG_HEAVY_NT 1024
#endif
// k_num_heavy_known geometry (rows-known units; default: the k_num_heavy geometry)
#ifndef CBG_KNOWN_LOGT
#define CBG_KNOWN_LOGT CBG_HEAVY_LOGT
#endif
#ifndef CBG_KNOWN_NT
#define CBG_KNOWN_NT CBG_HEAVY_NT
#endif
#ifndef CBG_ITEM_UNITS
#define CBG_ITEM_UNITS 4
#endif
// k_num_heavy rank mode: single-chunk units whose span fits a 32*T-row bitmap get exact slots
#ifndef CBG_RANK_MODE
#define CBG_RANK_MODE 1
#endif
// rank mode: register-resident sweeps for chunks of <= NT*U*CBG_RANK_REGS groups
#ifndef CBG_RANK_REGS
#define CBG_RANK_REGS 6
#endif
// units also end before their row span exceeds CBG_RANK_SPAN_CAP rows (0 = no span limit)
#ifndef CBG_RANK_SPAN_CAP
#define CBG_RANK_SPAN_CAP 458752   // f64, T=8192, NT=1024, unit cap 6144: <= (9216*12 - 6144*8)/4 words
#endif
#ifndef CBG_UNIT_CAP
// rank mode holds up to T outputs.  Round 5 measured 7/8 T best (s20 66.9 -> 66.3 ms, s21 203.4 -> 202.2 ms against
// 3/4 T; T faster at s20, slower at s21: profiles/r05s_unit_cap_ab.txt, r05t_unit_cap_ab.txt); with the adaptive unit
// span (round 6) T is ahead everywhere: s20 64.0 -> 63.7 ms, s21 194.7 -> 194.2 ms, s22 2x2x2 rank 0 81.2 -> 80.4 ms
// (3/4 T: 64.6 / 196.8 / 82.7 ms; profiles/r06m_unit_cap_ab.txt)
#define CBG_UNIT_CAP (1 << CBG_HEAVY_LOGT)
#endif
// smallest subwindow: 2^13 rows, or the heavy table's 2^CBG_HEAVY_LOGT when that is smaller (a one-subwindow unit
// must fit k_num_heavy's dense table)
constexpr int kSubLogMin = CBG_HEAVY_LOGT < 13 ? CBG_HEAVY_LOGT : 13;
constexpr int64_t kUnitCap = CBG_UNIT_CAP;   // max outputs of a multi-subwindow unit (load <= kUnitCap/T)
constexpr int kSplitMin = 16;      // A columns at least this long get split-table rows
constexpr int kMaxSub = 2048;      // max subwindows per column (SUBW chosen so nrow/SUBW <= kMaxSub)
constexpr int kItemUnits = CBG_ITEM_UNITS; // units of one heavy column per workgroup item (k_num_heavy)
constexpr int kMaxParts = 32;      // symbolic parts per wide column (wider, hypersparse columns: windowed path)

template <typename V>
struct DevCsc {
  int64_t nrow, ncol, nnz;
  const int64_t* cp;
  const int32_t* ir;
  const V* val;   // nullptr => pattern, all values 1/true
};

// split table: for long A columns, tab[idx[k]*(nsub+1) + s] = (first entry with row >= s*SUBW) - cp[k]
// symbolic -> numeric row handoff element: the whole row.  (A 16-bit form rebuilt from per-unit 2^16-row block thresholds
// halved the handoff bytes, s20 11.3 -> 5.6 GB, but the rebuild sat on the rows-known kernel's per-unit critical path:
// heavy 31.2 -> 35.0 ms, profiles/r05f_rows16_ab_s20.txt; removed in round 6, it lives in git history.)
typedef int32_t HRow;
struct UnitSeg;
struct UnitRows;
struct Split {
  const int32_t* idx;   // per A column: row of tab, or -1
  const int32_t* tab;
  int32_t nsub;         // subwindows in the row space
  int32_t log;          // log2(SUBW)
  const UnitSeg* useg;  // precomputed unit segments (k_unit_segs)
  const HRow* hrows;    // sorted output rows of heavy columns written by the symbolic pass (or null)
  const UnitRows* urows;// per unit: where its rows lie in hrows (k_build_units)
  const int32_t* ptab;  // part table (k_part_table): row k = [cp[k] (two words), then for p = 0..P: (first entry with
                        // row >= p*2^kPartLog) - cp[k]]
  int32_t pstride;      // words per row: a power of two >= parts + 3 (0: no table)
};

struct Unit {
  int32_t j;            // output column
  int32_t s0, s1;       // subwindows [s0, s1)
  int32_t cnt;          // outputs
  int64_t outoff;       // position of the first output in C
  int64_t segbase;      // this unit's A segments in the precomputed table (UnitSeg), or -1
};

struct UnitSeg {        // A segment [a0, a1) of one (unit, B nonzero) pair
  int64_t a0, a1;
};

// A unit's output rows inside the symbolic pass's row scratch: up to 3 contiguous pieces (a unit's
// span crosses at most two 2^kPartLog-row part boundaries); np = 0: rows unknown (old rank path).
struct UnitRows {
  int64_t off[3];
  int32_t n[3];
  int32_t np;
};

// per-item description shared by all numeric/symbolic kernels
struct Work {
  int32_t j;
  int32_t lo, hi;       // row range [lo, hi]
  int32_t s0, s1;       // unit subwindows, s0 < 0 for a whole column
  int64_t ob;           // output offset (numeric)
  int64_t segbase;      // unit: precomputed segments (index of B(:,j)'s first nonzero), or -1
};

template <typename V>
__device__ __forceinline__ V load_val(const V* v, int64_t i) { return v ? v[i] : V(1); }

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }

// Diagnostic build only (-DCBG_STAMPS, tools/diag): per-phase cycle sums of thread 0 of every
// workgroup, read back with cbg_debug_stamps.  No stamp executes in the product library.
#ifdef CBG_STAMPS
__device__ unsigned long long g_stamps[32];
#define STAMP_DECL unsigned long long st_prev_ = 0;
#define STAMP(i)                                                                        \
  do {                                                                                  \
    if (threadIdx.x == 0) {                                                             \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime();                       \
      if (st_prev_) atomicAdd(&g_stamps[i], t_ - st_prev_);                             \
      st_prev_ = t_;                                                                    \
    }                                                                                   \
  } while (0)
#define STAMP_COUNT(i, v) do { if (threadIdx.x == 0) atomicAdd(&g_stamps[i], (unsigned long long)(v)); } while (0)
#else
#define STAMP_DECL
#define STAMP(i) do {} while (0)
#define STAMP_COUNT(i, v) do {} while (0)
#endif

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
// DPP forms (GFX9 data-parallel primitives, no LDS crossbar): row_shr within 16-lane rows, then row_bcast:15 /
// row_bcast:31 carry the row totals across the wave.  Lanes whose source is out of range read `old` = 0.
__device__ __forceinline__ int dpp_incl_scan(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);   // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);   // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);   // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);   // row_shr:8
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);   // row_bcast:15 into rows 1, 3
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);   // row_bcast:31 into rows 2, 3
  return v;
}
__device__ __forceinline__ int64_t dpp_shift64(int64_t v, int ctrl_sel) {
  const uint32_t lo = (uint32_t)v, hi = (uint32_t)((uint64_t)v >> 32);
  uint32_t a, b;
  switch (ctrl_sel) {
    case 0: a = __builtin_amdgcn_update_dpp(0u, lo, 0x111, 0xf, 0xf, false); b = __builtin_amdgcn_update_dpp(0u, hi, 0x111, 0xf, 0xf, false); break;
    case 1: a = __builtin_amdgcn_update_dpp(0u, lo, 0x112, 0xf, 0xf, false); b = __builtin_amdgcn_update_dpp(0u, hi, 0x112, 0xf, 0xf, false); break;
    case 2: a = __builtin_amdgcn_update_dpp(0u, lo, 0x114, 0xf, 0xf, false); b = __builtin_amdgcn_update_dpp(0u, hi, 0x114, 0xf, 0xf, false); break;
    case 3: a = __builtin_amdgcn_update_dpp(0u, lo, 0x118, 0xf, 0xf, false); b = __builtin_amdgcn_update_dpp(0u, hi, 0x118, 0xf, 0xf, false); break;
    case 4: a = __builtin_amdgcn_update_dpp(0u, lo, 0x142, 0xa, 0xf, false); b = __builtin_amdgcn_update_dpp(0u, hi, 0x142, 0xa, 0xf, false); break;
    default: a = __builtin_amdgcn_update_dpp(0u, lo, 0x143, 0xc, 0xf, false); b = __builtin_amdgcn_update_dpp(0u, hi, 0x143, 0xc, 0xf, false); break;
  }
  return (int64_t)(((uint64_t)b << 32) | a);
}
__device__ __forceinline__ int64_t dpp_incl_scan64(int64_t v) {
#pragma unroll
  for (int k = 0; k < 6; ++k) v += dpp_shift64(v, k);
  return v;
}
// the value of lane l-1 (lane 0: 0): wave_shr:1
__device__ __forceinline__ uint32_t dpp_prev_lane(uint32_t v) {
  return __builtin_amdgcn_update_dpp(0u, v, 0x138, 0xf, 0xf, false);
}
// lane 63's value, uniform (scalar read)
__device__ __forceinline__ uint32_t last_lane(uint32_t v) { return __builtin_amdgcn_readlane(v, 63); }
__device__ __forceinline__ int64_t last_lane64(int64_t v) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, 63);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)((uint64_t)v >> 32), 63);
  return (int64_t)(((uint64_t)hi << 32) | lo);
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
  if (threadIdx.x < kWave) {
    const int p = l < NW ? scratch[l] : 0;
    const int pi = wave_incl_scan(p);
    if (l < NW) scratch[l] = pi - p;
    if (l == NW - 1) scratch[NW] = pi;
  }
  __syncthreads();
  int ex = scratch[w] + inc - v;
  *total = scratch[NW];
  __syncthreads();
  return ex;
}

// first position in [lo, hi) with ir[pos] >= r (ir ascending)
__device__ __forceinline__ int64_t lower_bound_rows(const int32_t* __restrict__ ir, int64_t lo, int64_t hi, int64_t r) {
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if ((int64_t)ir[mid] < r) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// A segment of unit (s0, s1) inside column k: exact for split-table columns; a short column
// (< kSplitMin entries) is taken whole and its rows outside the unit are dropped at insert time
// (cheaper than two dependent binary searches per unit and B nonzero).
__device__ __forceinline__ void unit_bounds(const int64_t* __restrict__ Acp, const Split& sp, int32_t k,
                                            int32_t s0, int32_t s1, int64_t& a0, int64_t& a1) {
  const int64_t c0 = Acp[k], c1 = Acp[k + 1];
  if (c1 - c0 >= kSplitMin) {
    const int32_t* t = sp.tab + (int64_t)sp.idx[k] * (sp.nsub + 1);
    a0 = c0 + t[s0];
    a1 = c0 + t[s1];
  } else {
    a0 = c0;
    a1 = c1;
  }
}

// ============================================================================ 1. column statistics
// Every A column's (length, first row, last row, split-table row or -1) in one 16-byte record, written by one streaming
// pass over A's column pointers: the statistics and the unit segment table gather one record per B nonzero instead of
// the two pointers, the first and last rows and the split index (up to four random cache lines; the 2^22 A columns of
// an s22 rank panel miss the L2 on most of them).  The same pass numbers the long columns (>= kSplitMin entries) for
// the split table: each workgroup takes a contiguous range of columns, counts its long ones, claims their numbers with
// ONE atomic, then numbers them in order -- a claim per wavefront serialised ~2^16 same-address atomics at the L2
// (k_split_assign: 0.74 ms for the 2^22 columns of a rank panel, 0.17 ms at s20).
__global__ void __launch_bounds__(256) k_acol_info(int64_t ncol, const int64_t* __restrict__ Acp,
                                                   const int32_t* __restrict__ Air, int4* __restrict__ info,
                                                   int32_t* __restrict__ idx, int32_t* __restrict__ longcols,
                                                   int* __restrict__ nlong) {
  __shared__ int s_w[256 / kWave];
  __shared__ int s_base;
  const int64_t per = (ncol + gridDim.x - 1) / gridDim.x;
  const int64_t c0 = blockIdx.x * per, c1 = min(ncol, c0 + per);
  const int lane = lane_id(), w = threadIdx.x / kWave;
  int cnt = 0;
  for (int64_t k = c0 + threadIdx.x; k < c1; k += 256) cnt += Acp[k + 1] - Acp[k] >= kSplitMin;
  cnt = (int)wave_sum64(cnt);
  if (lane == 0) s_w[w] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int v = 0; v < 256 / kWave; ++v) t += s_w[v];
    s_base = t ? atomicAdd(nlong, t) : 0;
  }
  __syncthreads();
  int run = s_base;
  for (int64_t t0 = c0; t0 < c1; t0 += 256) {
    const int64_t k = t0 + threadIdx.x;
    int64_t a0 = 0, a1 = 0;
    if (k < c1) { a0 = Acp[k]; a1 = Acp[k + 1]; }
    const bool lng = a1 - a0 >= kSplitMin;
    const uint64_t m = __ballot(lng);
    __syncthreads();   // s_w reused
    if (lane == 0) s_w[w] = __popcll(m);
    __syncthreads();
    int before = 0, tile = 0;
    for (int v = 0; v < 256 / kWave; ++v) {
      before += v < w ? s_w[v] : 0;
      tile += s_w[v];
    }
    if (k < c1) {
      const int e = lng ? run + before + __popcll(m & ((1ull << lane) - 1ull)) : -1;
      idx[k] = e;
      if (lng) longcols[e] = (int32_t)k;
      info[k] = a1 > a0 ? make_int4((int)(a1 - a0), Air[a0], Air[a1 - 1], e) : make_int4(0, INT32_MAX, -1, -1);
    }
    run += tile;
  }
}

// flop[j] = sum_{k in B(:,j)} nnz(A(:,k))   (estimateFLOP, mtSpGEMM.h:1117-1135)
// span[j] = [min, max] row index any of those A columns holds (A columns are row-sorted).
// LPC lanes per column (4, 8 or 16: the host picks the power of two nearest nnz(B)/ncol, so short columns do
// not idle most of a 16-lane group).
template <int LPC>
__global__ void __launch_bounds__(256) k_col_stats(int64_t ncol, const int4* __restrict__ ainfo,
                                                   const int64_t* __restrict__ Bcp,
                                                   const int32_t* __restrict__ Bir,
                                                   int64_t* __restrict__ flop, int2* __restrict__ span,
                                                   unsigned long long* __restrict__ total) {
  // LPC lanes per column, grid-stride over column groups; the block totals are added once per block
  // (one global atomic per block: a same-address atomic per column group serialised at the L2)
  constexpr int LOG = LPC == 4 ? 2 : LPC == 8 ? 3 : 4;
  static_assert(LPC == 4 || LPC == 8 || LPC == 16, "4, 8 or 16 lanes per column");
  const int sub = threadIdx.x & (LPC - 1);
  int64_t wf = 0, hb = 0;
  for (int64_t j = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> LOG; j < ncol;
       j += ((int64_t)gridDim.x * blockDim.x) >> LOG) {
    int64_t f = 0;
    int lo = INT32_MAX, hi = -1;
    const int64_t e = Bcp[j + 1];
    for (int64_t p = Bcp[j] + sub; p < e; p += LPC) {
      const int4 a = ainfo[Bir[p]];   // (length, first row, last row); an empty column: (0, INT32_MAX, -1)
      f += a.x;
      lo = min(lo, a.y);
      hi = max(hi, a.z);
    }
#pragma unroll
    for (int d = LPC / 2; d > 0; d >>= 1) {
      f += __shfl_xor(f, d, LPC);
      lo = min(lo, __shfl_xor(lo, d, LPC));
      hi = max(hi, __shfl_xor(hi, d, LPC));
    }
    if (sub == 0) {
      flop[j] = f;
      span[j] = make_int2(lo, hi);
      wf += f;
      // an upper bound of the heavy columns' outputs, sum of min(flop, span) over columns with
      // flop > kHeavy -> total[10] (row handoff scratch)
      if (f > 4096 && hi >= lo) hb += min(f, (int64_t)hi - lo + 1);
    }
  }
  __shared__ unsigned long long s_tot, s_hb;
  if (threadIdx.x == 0) { s_tot = 0; s_hb = 0; }
  __syncthreads();
  wf = wave_sum64(wf);
  hb = wave_sum64(hb);
  if (lane_id() == 0 && wf) atomicAdd(&s_tot, (unsigned long long)wf);
  if (lane_id() == 0 && hb) atomicAdd(&s_hb, (unsigned long long)hb);
  __syncthreads();
  if (threadIdx.x == 0 && s_tot) atomicAdd(total, s_tot);
  if (threadIdx.x == 0 && s_hb) atomicAdd(total + 10, s_hb);
}

// ============================================================================ 2. binning
// Class ids (shared by symbolic and numeric binning, different size meaning):
//   0              : empty item (nothing to do)
//   1..NWC         : wave classes, table T = 64 << (c-1)
//   NWC+1..NWC+NBC : block classes, table T = (64 << NWC) << (c-1-NWC)
//   NWC+NBC+1      : windowed (heavy) class
struct BinParams {
  int nwave, nblock;     // number of wave / block classes
  int64_t wave_min_T;    // 64
  int sym;               // 1: symbolic (need = min(2*flop, span words)); 0: numeric (need = min(2*nnz, span))
  int lane_max;          // columns with 0 < flop <= lane_max go to kLaneClass (one lane per column); 0 = off
};
constexpr int kLaneClass = 30;   // list class of the one-lane-per-column kernels (hist[30])
constexpr int kLaneMax = 16;     // their per-lane table size: flop <= kLaneMax
constexpr int kLane8Class = 29;  // numeric binning: flop <= kLaneSmall (half the per-lane LDS, twice the lanes per CU)
constexpr int kLaneSmall = 8;

__device__ __forceinline__ int class_of(int64_t need, const BinParams& bp) {
  if (need <= 0) return 0;
  int64_t T = bp.wave_min_T;
  const int ntot = bp.nwave + bp.nblock;
  for (int c = 1; c <= ntot; ++c, T <<= 1)
    if (need <= T) return c;
  return ntot + 1;
}

// symbolic bitmaps start at a 32-aligned row, hence the extra word
__device__ __forceinline__ int64_t need_of(int64_t cnt, int2 sp, int sym) {
  if (cnt <= 0 || sp.y < sp.x) return 0;
  const int64_t span = (int64_t)sp.y - sp.x + 1;
  if (sym) return min(2 * cnt, (int64_t)((sp.y - (sp.x & ~31)) >> 5) + 1);   // exact bitmap words
  return min(2 * cnt, span);
}

// pass 0: histogram; pass 1: scatter into class-contiguous list using device cursors.
// hist[31] counts items with cnt > heavy (capacity of the heavy lists).  Each block takes kBinPer
// consecutive items per thread, so the per-class global atomics are one per block per class (not one
// per 256 items: same-address atomics serialise at the L2).  flop (optional): lane-class test for the
// numeric binning, whose cnt is nnz(C(:,j)).
constexpr int kBinPer = 8;
__global__ void __launch_bounds__(256) k_bin(int64_t n, const int64_t* __restrict__ cnt,
                                             const int2* __restrict__ span, const int64_t* __restrict__ flop,
                                             BinParams bp, int pass, int64_t heavy,
                                             unsigned long long* __restrict__ hist,
                                             unsigned long long* __restrict__ cursor,
                                             int32_t* __restrict__ list) {
  __shared__ unsigned int s_h[32];
  __shared__ unsigned long long s_base[32];
  const int ncls = bp.nwave + bp.nblock + 2;
  if (threadIdx.x < 32) s_h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t j0 = (int64_t)blockIdx.x * blockDim.x * kBinPer;
  int cls[kBinPer];
  unsigned int rank[kBinPer];
#pragma unroll
  for (int r = 0; r < kBinPer; ++r) {
    const int64_t j = j0 + (int64_t)r * blockDim.x + threadIdx.x;
    cls[r] = -1;
    rank[r] = 0;
    if (j < n) {
      const int64_t cj = cnt[j];
      const int64_t fj = flop ? flop[j] : cj;
      const int c = (bp.lane_max > 0 && cj > 0 && fj <= bp.lane_max)
                        ? (!bp.sym && fj <= kLaneSmall ? kLane8Class : kLaneClass)
                        : class_of(need_of(cj, span[j], bp.sym), bp);
      cls[r] = c;
      rank[r] = atomicAdd(&s_h[c], 1u);
      if (pass == 0 && cj > heavy) atomicAdd(&s_h[31], 1u);
    }
  }
  __syncthreads();
  const bool used = threadIdx.x < ncls || threadIdx.x == kLaneClass || threadIdx.x == kLane8Class;
  if (pass == 0) {
    if ((used || threadIdx.x == 31) && s_h[threadIdx.x])
      atomicAdd(&hist[threadIdx.x], (unsigned long long)s_h[threadIdx.x]);
    return;
  }
  // the class offsets from pass 0's totals, laid out as bin_fill's host copy (the regular classes in order, then
  // the lane classes), so that no host-to-device copy sits between the passes; cursor starts at zero
  if (threadIdx.x == 0) {
    unsigned long long h[32];
#pragma unroll
    for (int c = 0; c < 32; ++c) h[c] = hist[c];
    unsigned long long acc = 0;
    for (int c = 0; c < ncls; ++c) { s_base[c] = acc; acc += h[c]; }
    s_base[kLane8Class] = acc;
    s_base[kLaneClass] = acc + h[kLane8Class];
  }
  __syncthreads();
  if (used && s_h[threadIdx.x])
    s_base[threadIdx.x] += atomicAdd(&cursor[threadIdx.x], (unsigned long long)s_h[threadIdx.x]);
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kBinPer; ++r)
    if (cls[r] >= 0) list[s_base[cls[r]] + rank[r]] = (int32_t)(j0 + (int64_t)r * blockDim.x + threadIdx.x);
}

// ============================================================================ one-lane columns
// Columns with at most kLaneMax multiplies (e.g. R^T A with an aggregation R: one multiply per A
// entry) get one LANE each instead of a wavefront: the lane walks its few (B nonzero, A entry) pairs
// into a private LDS slice, counts (symbolic) or accumulates, sorts and writes (numeric).  A wave
// per such column spent its time on table set-up and scans for a handful of multiplies.
constexpr int kLaneStride = kLaneMax + 1;   // odd stride: the 64 lanes' slices start in distinct banks
constexpr int kLaneBatch = 8;               // B nonzeros whose loads a lane issues together

__global__ void __launch_bounds__(256) k_sym_lane(const int32_t* __restrict__ list, int64_t count,
                                                  const int64_t* __restrict__ Acp, const int32_t* __restrict__ Air,
                                                  const int64_t* __restrict__ Bcp, const int32_t* __restrict__ Bir,
                                                  int64_t* __restrict__ nnz) {
  __shared__ int32_t s_rows[256 * kLaneStride];
  int32_t* rows = s_rows + threadIdx.x * kLaneStride;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < count; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t j = list[i];
    int m = 0;
    const int64_t bs = Bcp[j], be = Bcp[j + 1];
    for (int64_t b0 = bs; b0 < be; b0 += kLaneBatch) {   // batched independent loads, as k_num_lane
      int32_t k[kLaneBatch];
      int64_t a0[kLaneBatch], a1[kLaneBatch];
      int32_t r0[kLaneBatch];
#pragma unroll
      for (int t = 0; t < kLaneBatch; ++t) k[t] = b0 + t < be ? Bir[b0 + t] : 0;
#pragma unroll
      for (int t = 0; t < kLaneBatch; ++t) {
        const bool ok = b0 + t < be;
        a0[t] = ok ? Acp[k[t]] : 0;
        a1[t] = ok ? Acp[k[t] + 1] : 0;
      }
#pragma unroll
      for (int t = 0; t < kLaneBatch; ++t) r0[t] = a1[t] > a0[t] ? Air[a0[t]] : 0;
#pragma unroll
      for (int t = 0; t < kLaneBatch; ++t) {
        if (a1[t] <= a0[t] || m >= kLaneMax) continue;
        rows[m++] = r0[t];
        for (int64_t q = a0[t] + 1; q < a1[t] && m < kLaneMax; ++q) rows[m++] = Air[q];
      }
    }
    int d = 0;   // an entry counts when no earlier entry has its row
    for (int x = 0; x < m; ++x) {
      const int32_t r = rows[x];
      bool dup = false;
      for (int y = 0; y < x; ++y) dup |= rows[y] == r;
      d += !dup;
    }
    nnz[j] = d;
  }
}

// ============================================================================ segment expansion
// Visit every multiply of a work item: q in the A segment of b, for b in B(:,j)[bs, be).  The B
// nonzeros are taken NT at a time (a wavefront when WAVE, else the block); each lane computes its
// segment (seg(b, a0, a1, bv)), a scan over the segment lengths gives every multiply a flat index
// m, and then the NT lanes take consecutive m's: lane t handles m = m0 + u*NT + t and finds its
// segment by a binary search over the LDS prefix offsets.  Every lane gets the same share of the
// multiplies whatever the (power-law) segment lengths, consecutive lanes read consecutive A
// entries of one segment (coalesced), and each lane keeps U independent gathers in flight.
// ld(q) loads what an insert needs; ins(item, bv, q, b) inserts it.
// A row loader with a 16-byte path: expand_staged issues ONE global_load_dwordx4 (4-byte alignment suffices on
// gfx950) for a lane's group of 4 consecutive A entries instead of four dword loads.  Near the end of A.ir the
// load is moved back to stay in bounds and the entries shifted (the group's entries beyond its segment are
// never inserted, so what they hold does not matter; only the array end needs care).
typedef int32_t cbg_v4i __attribute__((ext_vector_type(4)));
struct RowLd4 {
  const int32_t* ir;
  int64_t n;   // entries of A (>= 4 for the vector path)
  __device__ __forceinline__ int32_t operator()(int64_t q) const { return ir[q]; }
  __device__ __forceinline__ cbg_v4i vec4(int64_t q) const {
    const int64_t qv = q + 4 <= n ? q : n - 4;
    cbg_v4i v;
    __builtin_memcpy(&v, ir + qv, 16);
    const int d = (int)(q - qv);
    if (d == 1) v = cbg_v4i{v.y, v.z, v.w, v.w};
    else if (d == 2) v = cbg_v4i{v.z, v.w, v.w, v.w};
    else if (d == 3) v = cbg_v4i{v.w, v.w, v.w, v.w};
    return v;
  }
};
template <class F> struct HasVec4 { static constexpr bool value = false; };
template <> struct HasVec4<RowLd4> { static constexpr bool value = true; };
template <class F> struct HasVec2 { static constexpr bool value = false; };   // (row, value) pairs: NumLd2

template <typename V, typename IX = int64_t>
struct SegBuf {         // LDS, NT entries each (+ scan scratch for block mode)
  IX* qb;               // segment start (A index)
  IX* off;              // exclusive prefix of segment group counts of one chunk (bounded: see k_sym_part)
  V* bv;                // B value of the segment's nonzero
  int64_t* scratch;     // block mode: NT/64 + 1 entries
  int32_t* len;         // segment length (multiplies)
};

__device__ __forceinline__ int64_t wave_incl_scan64(int64_t v) {
  const int l = lane_id();
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const int64_t t = __shfl_up(v, d, kWave);
    if (l >= d) v += t;
  }
  return v;
}

// exclusive scan over the block (int64); the caller synchronises before `scratch` is reused
template <int NT>
__device__ __forceinline__ int64_t block_excl_scan64(int64_t v, int64_t* scratch, int64_t* total) {
  constexpr int NW = NT / kWave;
  const int w = threadIdx.x / kWave, l = lane_id();
  const int64_t inc = wave_incl_scan64(v);
  if (l == kWave - 1) scratch[w] = inc;
  __syncthreads();
  if (threadIdx.x < kWave) {
    const int64_t p = l < NW ? scratch[l] : 0;
    const int64_t pi = wave_incl_scan64(p);
    if (l < NW) scratch[l] = pi - p;
    if (l == NW - 1) scratch[NW] = pi;
  }
  __syncthreads();
  *total = scratch[NW];
  return scratch[w] + inc - v;
}

// s_waitcnt vmcnt(0) (expcnt/lgkmcnt left at their maxima; gfx9 encoding)
__device__ __forceinline__ void wait_vmem_all() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// last s in [0, P) with off[s] <= m (off non-decreasing, off[0] = 0 <= m): the non-empty segment
// holding flat multiply m.  P is a power of two covering the staged segments (P <= NT).
template <int NT, typename IX>
__device__ __forceinline__ int seg_search(const IX* off, int64_t m, int P) {
  int s = 0;
  for (int step = P >> 1; step > 0; step >>= 1)
    if (off[s + step] <= m) s += step;
  return s;
}

// U searches in lockstep: each step issues the U independent LDS reads together (one latency per
// step instead of U); steps >= P are skipped by a uniform branch.
template <int NT, int U, typename IX>
__device__ __forceinline__ void seg_search_n(const IX* off, const int64_t (&m)[U], int P, int (&s)[U]) {
#pragma unroll
  for (int u = 0; u < U; ++u) s[u] = 0;
#pragma unroll
  for (int step = NT >> 1; step > 0; step >>= 1) {
    if (step < P) {
      int64_t o[U];
#pragma unroll
      for (int u = 0; u < U; ++u) o[u] = off[s[u] + step];
#pragma unroll
      for (int u = 0; u < U; ++u) s[u] = o[u] <= m[u] ? s[u] + step : s[u];
    }
  }
}

// Stage one chunk of NT segments (this lane's a0, a1, bv) into LDS; returns the chunk's number of
// GROUPS: a segment of len multiplies is cut into ceil(len/G) groups of G consecutive A
// entries, and the groups (not the multiplies) are what lanes are dealt.  The LDS arrays are valid
// on return (synchronised).
template <int NT, bool WAVE, int G, typename V, typename IX>
__device__ __forceinline__ int64_t stage_segments(const SegBuf<V, IX>& sb, int64_t a0, int64_t a1, V bv) {
  const int tid = WAVE ? lane_id() : (int)threadIdx.x;
  const int64_t len = a1 - a0;
  const int64_t ng = (len + G - 1) / G;
  int64_t ex, F;
  if constexpr (WAVE) {
    const int64_t inc = wave_incl_scan64(ng);
    F = __shfl(inc, kWave - 1, kWave);
    ex = inc - ng;
  } else {
    ex = block_excl_scan64<NT>(ng, sb.scratch, &F);
  }
  sb.qb[tid] = (IX)a0;
  sb.off[tid] = (IX)ex;
  sb.len[tid] = (int32_t)len;
  sb.bv[tid] = bv;
  if constexpr (WAVE) wave_sync(); else __syncthreads();
  return F;
}

// Deal the F staged groups to the NT lanes: lane t takes groups g = g0 + u*NT + t and finds the
// group's segment by a binary search over the LDS prefix offsets (one search per G multiplies),
// then issues the group's G gathers back to back (U*G independent gathers per lane).
// `base` is the B position of staged segment 0.  The caller synchronises before re-staging.
template <int NT, int U, int G, typename V, class LdF, class InsF, typename IX>
__device__ __forceinline__ void expand_staged(const SegBuf<V, IX>& sb, int tid, int64_t F, int64_t base, int nseg,
                                              LdF ld, InsF ins) {
  using Item = decltype(ld(int64_t(0)));
  int P = 1;
  while (P < nseg) P <<= 1;
  for (int64_t g0 = 0; g0 < F; g0 += (int64_t)NT * U) {
    Item it[U][G];
    int ss[U];
    int64_t qq[U], m[U];
    int nv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t g = g0 + (int64_t)u * NT + tid;
      m[u] = g < F ? g : 0;
    }
    seg_search_n<NT, U>(sb.off, m, P, ss);
    // every load is issued unconditionally (index clamped into the group, or 0 for an idle lane, a
    // valid entry of any non-empty A): divergent conditional loads make the compiler drain the load
    // counter before each one, serialising the gathers
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int sg = ss[u];
      const int64_t k0 = (m[u] - sb.off[sg]) * G;
      qq[u] = sb.qb[sg] + k0;
      nv[u] = g0 + (int64_t)u * NT + tid < F ? (int)min<int64_t>(G, sb.len[sg] - k0) : 0;
      const int64_t qs = nv[u] > 0 ? qq[u] : 0;
      const int last = nv[u] > 0 ? nv[u] - 1 : 0;
      if constexpr (G == 4 && HasVec4<LdF>::value) {
        const cbg_v4i x = ld.vec4(qs);
        it[u][0] = x.x; it[u][1] = x.y; it[u][2] = x.z; it[u][3] = x.w;
      } else {
#pragma unroll
        for (int i = 0; i < G; ++i) it[u][i] = ld(qs + min(i, last));
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (nv[u] > 0) {
        const V bv = sb.bv[ss[u]];
#pragma unroll
        for (int i = 0; i < G; ++i)
          if (i < nv[u]) ins(it[u][i], bv, qq[u] + i, base + ss[u]);
      }
    }
  }
}

// expand_staged for an accumulator whose slot lookup only READS LDS (the rank directory): all U*G
// slots are looked up first (slotf, branch-free on the clamped items; < 0 = drop), so their LDS reads
// issue together, then the U*G accumulations run.
template <int NT, int U, int G, typename V, class LdF, class SlotF, class AccF, typename IX>
__device__ __forceinline__ void expand_staged_slots(const SegBuf<V, IX>& sb, int tid, int64_t F, int64_t base, int nseg,
                                                    LdF ld, SlotF slotf, AccF acc) {
  using Item = decltype(ld(int64_t(0)));
  int P = 1;
  while (P < nseg) P <<= 1;
  for (int64_t g0 = 0; g0 < F; g0 += (int64_t)NT * U) {
    Item it[U][G];
    int ss[U], sl[U][G];
    int64_t qq[U], m[U];
    int nv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t g = g0 + (int64_t)u * NT + tid;
      m[u] = g < F ? g : 0;
    }
    seg_search_n<NT, U>(sb.off, m, P, ss);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int sg = ss[u];
      const int64_t k0 = (m[u] - sb.off[sg]) * G;
      qq[u] = sb.qb[sg] + k0;
      nv[u] = g0 + (int64_t)u * NT + tid < F ? (int)min<int64_t>(G, sb.len[sg] - k0) : 0;
      const int64_t qs = nv[u] > 0 ? qq[u] : 0;
      const int last = nv[u] > 0 ? nv[u] - 1 : 0;
      if constexpr (G == 2 && HasVec2<LdF>::value) {
        ld.vec2(qs, it[u][0], it[u][1]);
      } else {
#pragma unroll
        for (int i = 0; i < G; ++i) it[u][i] = ld(qs + min(i, last));
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int i = 0; i < G; ++i) {
        const int v = slotf(it[u][i]);
        sl[u][i] = i < nv[u] ? v : -1;
      }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (nv[u] > 0) {
        const V bv = sb.bv[ss[u]];
#pragma unroll
        for (int i = 0; i < G; ++i)
          if (sl[u][i] >= 0) acc(sl[u][i], it[u][i], bv, qq[u] + i, base + ss[u]);
      }
    }
    // the gathers of a skipped accumulation were never waited on: drain them here, so the next round
    // (and a loop entered with prefetches in flight) does not start with a full memory-counter wait
    wait_vmem_all();
  }
}

// Two sweeps over one staged chunk (F <= NT*U*RI groups) with the row ids kept in registers:
// sweep 1 gathers the rows (ldr) and mark(row)s them; mid() (block-uniform: barrier + whatever must
// see all marks; false aborts); sweep 2 gathers the values (ldv) and acc(row, value, bv, q, b)s --
// the rank mode's two sweeps with each A entry's row and value gathered once.  Only the rows and a
// packed (segment, count) word per group stay live across mid(); q is recomputed from LDS.
template <int NT, int U, int G, int RI, typename V, class LdR, class LdV, class MarkF, class MidF, class AccF,
          typename IX>
__device__ __forceinline__ bool expand_staged_twice(const SegBuf<V, IX>& sb, int tid, int64_t F, int64_t base, int nseg,
                                                    LdR ldr, LdV ldv, MarkF mark, MidF mid, AccF acc) {
  int P = 1;
  while (P < nseg) P <<= 1;
  int32_t rr[RI][U][G];
  int sn[RI][U];   // segment << 8 | count (count <= G), 0 = no group
#pragma unroll
  for (int r = 0; r < RI; ++r)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t g = (int64_t)(r * U + u) * NT + tid;
      sn[r][u] = 0;
      if (g < F) {
        const int sg = seg_search<NT>(sb.off, g, P);
        const int64_t k0 = (g - sb.off[sg]) * G;
        const int64_t q = sb.qb[sg] + k0;
        const int nv = (int)min<int64_t>(G, sb.len[sg] - k0);
        sn[r][u] = (sg << 8) | nv;
#pragma unroll
        for (int i = 0; i < G; ++i)
          if (i < nv) rr[r][u][i] = ldr(q + i);
      }
    }
#pragma unroll
  for (int r = 0; r < RI; ++r)
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int i = 0; i < G; ++i)
        if (i < (sn[r][u] & 0xff)) mark(rr[r][u][i]);
  if (!mid()) return false;
#pragma unroll
  for (int r = 0; r < RI; ++r)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int nv = sn[r][u] & 0xff;
      if (nv > 0) {
        const int sg = sn[r][u] >> 8;
        const int64_t g = (int64_t)(r * U + u) * NT + tid;
        const int64_t q = sb.qb[sg] + (g - sb.off[sg]) * G;
        const V bv = sb.bv[sg];
        V av[G];
#pragma unroll
        for (int i = 0; i < G; ++i)
          if (i < nv) av[i] = ldv(q + i);
#pragma unroll
        for (int i = 0; i < G; ++i)
          if (i < nv) acc(rr[r][u][i], av[i], bv, q + i, base + sg);
      }
    }
  return true;
}

template <int NT, bool WAVE, int U, int G, typename V, class SegF, class LdF, class InsF, typename IX>
__device__ __forceinline__ void for_each_multiply(int64_t bs, int64_t be, SegBuf<V, IX> sb, SegF seg, LdF ld, InsF ins) {
  const int tid = WAVE ? lane_id() : (int)threadIdx.x;
  for (int64_t base = bs; base < be; base += NT) {
    const int64_t b = base + tid;
    int64_t a0 = 0, a1 = 0;
    V bv = V(0);
    if (b < be) seg(b, a0, a1, bv);
    const int64_t F = stage_segments<NT, WAVE, G, V>(sb, a0, a1, bv);
    expand_staged<NT, U, G, V>(sb, tid, F, base, (int)min<int64_t>(NT, be - base), ld, ins);
    if constexpr (WAVE) wave_sync(); else __syncthreads();
  }
}

// ============================================================================ accumulation helpers
template <typename Acc>
struct Table {
  int32_t* keys;   // hash: keys[Tcap]; dense: presence bitmap (T/32 words)
  Acc* vals;       // T (dense) or Tcap (hash) slots
  int32_t T;       // home range (hash) / rows (dense)
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
    // one LDS op per probe step: claims an empty slot, or returns the key already there
    const int32_t cur = atomicCAS(&t.keys[s], kEmpty, r);
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

// ============================================================================ 3. symbolic
// Exact nnz of C(:,j) (estimateNNZ_Hash, mtSpGEMM.h:866-933).  Mode per column: presence bitmap over
// the column's row span (from a 32-aligned base) when it fits the table, else a keys-only hash with
// T >= 2*flop.
struct HeavyOut {       // columns with nnz > kHeavy: list + nnz per subwindow
  int* n;
  int32_t* cols;
  int32_t* sub;         // [h * nsub + s]
  int32_t nsub, log;
  // Row handoff to the numeric pass (rows == nullptr: off).  A heavy column's bitmap is compacted
  // into its sorted output rows, written to `rows` at an offset reserved from `cursor` (capacity `cap`,
  // an upper bound of the heavy outputs); poff[h * kMaxParts + p] = offset of relative part p (or of
  // the whole column, p = 0); mode[h] = 1 whole column in one run, 2 per part, other = unavailable.
  HRow* rows;
  unsigned long long* cursor;
  unsigned long long cap;
  int64_t* poff;
  int32_t* mode;
  int64_t chunk;        // k_sym_part: rows reserved per workgroup at a time (0: one reservation per part)
};

__device__ __forceinline__ int64_t reserve_rows(const HeavyOut& ho, int64_t n) {
  const unsigned long long o = atomicAdd(ho.cursor, (unsigned long long)n);
  return (o + (unsigned long long)n <= ho.cap) ? (int64_t)o : -1;
}

// symbolic insert of row r into a presence bitmap (base = 32-aligned first row) or a keys-only hash;
// returns 1 if r is new
template <int LOGT>
__device__ __forceinline__ int sym_insert(int32_t* tab, bool bitmap, int32_t base, int32_t r) {
  if (bitmap) {
    const int32_t o = r - base;
    const uint32_t bit = 1u << (o & 31);
    if (tab[o >> 5] & bit) return 0;
    return (atomicOr((uint32_t*)&tab[o >> 5], bit) & bit) ? 0 : 1;
  }
  return hash_insert_sym(tab, r, LOGT);
}

template <int LOGT>
__global__ void __launch_bounds__(256) k_sym_wave(const int32_t* __restrict__ list, int64_t count,
                                                  const int64_t* __restrict__ Acp, const int32_t* __restrict__ Air,
                                                  const int64_t* __restrict__ Bcp, const int32_t* __restrict__ Bir,
                                                  const int2* __restrict__ span, int64_t* __restrict__ nnz,
                                                  HeavyOut ho) {
  constexpr int T = 1 << LOGT;
  __shared__ int32_t s_tab[4][T];
  __shared__ int64_t s_qb[4][kWave], s_off[4][kWave];
  __shared__ uint8_t s_bv[4][kWave];
  __shared__ int32_t s_len[4][kWave];
  const int w = threadIdx.x / kWave, l = lane_id();
  int32_t* tab = s_tab[w];
  const SegBuf<uint8_t> sb{s_qb[w], s_off[w], s_bv[w], nullptr, s_len[w]};
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  for (int64_t i = blockIdx.x * 4 + w; i < count; i += nwaves) {
    const int32_t j = list[i];
    const int2 sp = span[j];
    const int32_t base = sp.x & ~31;
    const bool bitmap = ((sp.y - base) >> 5) + 1 <= T;
    for (int s = l; s < T; s += kWave) tab[s] = bitmap ? 0 : kEmpty;
    wave_sync();
    int cnt = 0;
    for_each_multiply<kWave, true, kUnrollSym, kGroupSym, uint8_t>(
        Bcp[j], Bcp[j + 1], sb,
        [&](int64_t b, int64_t& a0, int64_t& a1, uint8_t&) {
          const int32_t k = Bir[b];
          a0 = Acp[k];
          a1 = Acp[k + 1];
        },
        [&](int64_t q) { return Air[q]; },
        [&](int32_t r, uint8_t, int64_t, int64_t) { cnt += sym_insert<LOGT>(tab, bitmap, base, r); });
    int64_t tot = wave_sum64(cnt);
    if (l == 0) nnz[j] = tot;
    if (tot > kHeavy) {
      // only a bitmap table can hold more than kHeavy rows (a hash of T <= 1024 keys holds <= 512):
      // register the column as heavy and count its rows per subwindow, like k_sym_block
      int h = 0;
      if (l == 0) {
        h = atomicAdd(ho.n, 1);
        ho.cols[h] = j;
      }
      h = __shfl(h, 0, kWave);
      const int32_t sf = sp.x >> ho.log, sl = sp.y >> ho.log;
      const int nw = ((sp.y - base) >> 5) + 1;
      int32_t* dst = ho.sub + (int64_t)h * ho.nsub;
      for (int32_t s = sf; s <= sl; ++s) {
        int c = 0;
        for (int w2 = l; w2 < nw; w2 += kWave)
          if (((base + 32 * w2) >> ho.log) == s) c += __popc((uint32_t)tab[w2]);
        const int64_t cs = wave_sum64(c);
        if (l == 0) dst[s] = (int32_t)cs;
      }
      if (ho.rows) {   // sorted rows for the numeric pass: words in order, 64 at a time
        int64_t off = 0;
        if (l == 0) off = reserve_rows(ho, tot);
        off = __shfl(off, 0, kWave);
        if (off >= 0) {
          int64_t run = off;
          for (int w0 = 0; w0 < nw; w0 += kWave) {
            const int w2 = w0 + l;
            uint32_t wd = w2 < nw ? (uint32_t)tab[w2] : 0u;
            const int pc = __popc(wd);
            const int inc = wave_incl_scan(pc);
            int64_t pos = run + inc - pc;
            while (wd) {
              const int b = __ffs(wd) - 1;
              wd &= wd - 1;
              ho.rows[pos++] = (HRow)(base + 32 * w2 + b);
            }
            run += __shfl(inc, kWave - 1, kWave);
          }
        }
        if (l == 0) {
          ho.poff[(int64_t)h * kMaxParts] = off;
          ho.mode[h] = off >= 0 ? 1 : 0;
        }
      }
    }
    wave_sync();
  }
}

// block kernel: one column per workgroup; heavy columns also report nnz per subwindow
template <int LOGT, int NT>
constexpr size_t sym_block_lds() {
  return (size_t)(1 << LOGT) * 4 + (size_t)NT * 21 + (size_t)(NT / kWave + 1) * 8 + (size_t)(kMaxSub + 2) * 4 + 64;
}

template <int LOGT, int NT>
__global__ void __launch_bounds__(NT) k_sym_block(const int32_t* __restrict__ list, int64_t count,
                                                  const int64_t* __restrict__ Acp, const int32_t* __restrict__ Air,
                                                  const int64_t* __restrict__ Bcp, const int32_t* __restrict__ Bir,
                                                  const int2* __restrict__ span, int64_t* __restrict__ nnz,
                                                  HeavyOut ho) {
  constexpr int T = 1 << LOGT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int64_t* qb = (int64_t*)smem;                   // NT
  int64_t* off = qb + NT;                         // NT
  int64_t* scr = off + NT;                        // NT/64 + 1
  int32_t* tab = (int32_t*)(scr + NT / kWave + 1);// T
  int32_t* scnt = tab + T;                        // kMaxSub + 2
  int* misc = scnt + kMaxSub + 2;                 // [1] total, [2] heavy id
  int32_t* lens = misc + 8;                       // NT
  uint8_t* bvs = (uint8_t*)(lens + NT);           // NT
  const SegBuf<uint8_t> sb{qb, off, bvs, scr, lens};
  for (int64_t i = blockIdx.x; i < count; i += gridDim.x) {
    const int32_t j = list[i];
    const int2 sp = span[j];
    const int32_t base = sp.x & ~31;
    const bool bitmap = ((sp.y - base) >> 5) + 1 <= T;
    for (int s = threadIdx.x; s < T; s += NT) tab[s] = bitmap ? 0 : kEmpty;
    if (threadIdx.x == 0) misc[1] = 0;
    __syncthreads();
    int cnt = 0;
    for_each_multiply<NT, false, kUnrollSym, kGroupSym, uint8_t>(
        Bcp[j], Bcp[j + 1], sb,
        [&](int64_t b, int64_t& a0, int64_t& a1, uint8_t&) {
          const int32_t k = Bir[b];
          a0 = Acp[k];
          a1 = Acp[k + 1];
        },
        [&](int64_t q) { return Air[q]; },
        [&](int32_t r, uint8_t, int64_t, int64_t) { cnt += sym_insert<LOGT>(tab, bitmap, base, r); });
    int64_t wc = wave_sum64(cnt);
    if (lane_id() == 0 && wc) atomicAdd(&misc[1], (int)wc);
    __syncthreads();
    const int total = misc[1];
    if (threadIdx.x == 0) nnz[j] = total;
    if (total > kHeavy) {   // uniform branch
      const int32_t sf = sp.x >> ho.log, sl = sp.y >> ho.log;
      if (threadIdx.x == 0) {
        const int h = atomicAdd(ho.n, 1);
        misc[2] = h;
        ho.cols[h] = j;
      }
      for (int s = threadIdx.x; s <= sl - sf; s += NT) scnt[s] = 0;
      __syncthreads();
      if (bitmap) {
        const int nw = ((sp.y - base) >> 5) + 1;
        for (int w = threadIdx.x; w < nw; w += NT) {
          const uint32_t word = (uint32_t)tab[w];
          if (word) atomicAdd(&scnt[((base + 32 * w) >> ho.log) - sf], __popc(word));
        }
      } else {
        for (int s = threadIdx.x; s < T; s += NT) {
          const int32_t key = tab[s];
          if (key != kEmpty) atomicAdd(&scnt[(key >> ho.log) - sf], 1);
        }
      }
      __syncthreads();
      int32_t* dst = ho.sub + (int64_t)misc[2] * ho.nsub;
      for (int s = threadIdx.x; s <= sl - sf; s += NT) dst[sf + s] = scnt[s];
      if (ho.rows && bitmap) {   // sorted rows for the numeric pass: contiguous words per thread
        const int nw = ((sp.y - base) >> 5) + 1;
        const int WPT = (nw + NT - 1) / NT;
        const int w0 = min(nw, (int)threadIdx.x * WPT), w1 = min(nw, w0 + WPT);
        int c = 0;
        for (int w = w0; w < w1; ++w) c += __popc((uint32_t)tab[w]);
        int tot2;
        const int ex = block_excl_scan<NT>(c, lens, &tot2);   // lens is idle after the expansion
        if (threadIdx.x == 0) {
          const int64_t off = reserve_rows(ho, tot2);
          misc[4] = (int)(off & 0xffffffff);
          misc[5] = (int)(off >> 32);
          ho.poff[(int64_t)misc[2] * kMaxParts] = off;
          ho.mode[misc[2]] = off >= 0 ? 1 : 0;
        }
        __syncthreads();
        const int64_t off = (int64_t)(uint32_t)misc[4] | ((int64_t)misc[5] << 32);
        if (off >= 0) {
          int64_t pos = off + ex;
          for (int w = w0; w < w1; ++w) {
            uint32_t wd = (uint32_t)tab[w];
            while (wd) {
              const int b = __ffs(wd) - 1;
              wd &= wd - 1;
              ho.rows[pos++] = (HRow)(base + 32 * w + b);
            }
          }
        }
      }
    }
    __syncthreads();
  }
}

// Wide columns (bitmap > 16384 words): the row space is cut into aligned parts of 2^kPartLog rows and
// each (column, part) is one work item with a 64 KB bitmap, so two workgroups share a CU and hide
// each other's gather latency (one 128 KB bitmap per CU left the CU idle on every dependent load).
// A long A column contributes only its entries inside the part (split table, exact); a short one is
// read whole and filtered at insert.  Every wide column is registered as heavy up front; its parts
// write disjoint subwindow counts and add their totals into nnz[j].
#ifndef CBG_PART_LOG
#define CBG_PART_LOG 18
#endif
#ifndef CBG_PART_NT
#define CBG_PART_NT 512
#endif
constexpr int kPartLog = CBG_PART_LOG;
constexpr int kPartNT = CBG_PART_NT;
// persistent heavy kernels take their work from a device ticket (CBG_HEAVY_DYNAMIC=1) instead of a static stride:
// a workgroup that starts late -- its CU held by another stream's kernel, e.g. RCCL's fiber transfer (37.6 KB of LDS
// per workgroup) -- finds the work taken instead of holding a fixed share until the other kernel ends
#ifndef CBG_HEAVY_DYNAMIC
#define CBG_HEAVY_DYNAMIC 1
#endif
// Measured and removed (round 6; the variants live in git history): k_num_heavy_known computing its unit segments from
// the split table (r03t: heavy +8 ms); k_sym_part narrowing a short A column by binary search (r03s: +0.8 ms), emitting
// its rows word-major per wave (r03d), staging the next part's first chunk across the current one (r05d: +0.5 ms) and
// sweeping every part of a column in one workgroup (r05k: +1.4 ms).
#ifndef CBG_SYM_TESTOR
#define CBG_SYM_TESTOR 1   // k_sym_part reads a bitmap word before setting a bit (0: no-return ds_or only)
#endif
#ifndef CBG_SYM_ROWS_LDS
#define CBG_SYM_ROWS_LDS 1 // k_sym_part stages a part's rows in its (then idle) bitmap LDS and stores them coalesced (s20 symbolic 21.6 -> 20.7 ms, profiles/r05h_rows_lds_ab.txt; 0: each thread stores its own rows)
#endif
// first symbolic class (LOGT = class + 5) cut into parts: bitmaps larger than one part; every such
// column has flop > kHeavy (2*flop > 2^(class+4) words), so the heavy lists can hold it
constexpr int kWideClass = kPartLog - 9 > 9 ? kPartLog - 9 : 9;
static_assert(kPartLog >= 17 && kPartLog <= 19, "part bitmap 16..64 KB");
struct PartItem {
  int32_t j, p, h;
};

__global__ void k_part_items(const int32_t* __restrict__ list, int64_t count, int maxparts, const int2* __restrict__ span,
                             HeavyOut ho, PartItem* __restrict__ items, int* __restrict__ nitems,
                             int32_t* __restrict__ wlist, int* __restrict__ nwin) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < count; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t j = list[i];
    const int2 sp = span[j];
    const int np = (sp.y >> kPartLog) - (sp.x >> kPartLog) + 1;
    if (np <= maxparts) {
      const int h = atomicAdd(ho.n, 1);
      ho.cols[h] = j;
      const int e = atomicAdd(nitems, np);
      for (int p = 0; p < np; ++p) items[e + p] = PartItem{j, p, h};
    } else {
      wlist[atomicAdd(nwin, 1)] = j;
    }
  }
}

// Segment staging of k_sym_part: 32-bit (A.nnz < 2^31: segment starts are A positions; the group offsets of a chunk
// stay below NT * 2^kPartLog / kGroupSym <= 2^25 whatever B holds -- a segment is one A column narrowed to one part,
// at most 2^kPartLog entries since A's rows ascend strictly -- so repeated rows in a B column cannot overflow) lets four 512-thread workgroups share a CU's LDS and the kernel run at <= 64 VGPRs: 8 waves per
// SIMD instead of 6 (s20 symbolic 23.4 -> 22.1 ms, s21 80.5 -> 75.8 ms, profiles/r04e_*); 64-bit otherwise.
static_assert(((int64_t)kPartNT << kPartLog) < INT32_MAX,
              "a chunk's staged multiplies (NT segments of <= 2^kPartLog entries each) fit 32-bit offsets");
template <int NT, typename IX>
constexpr size_t sym_part_lds() {
  return (size_t)(1 << (kPartLog - 5)) * 4 + (size_t)NT * (2 * sizeof(IX) + 5) + (size_t)(NT / kWave + 1) * 8 +
         (size_t)((1 << (kPartLog - kSubLogMin)) + 8) * 4 + 64;
}

template <int NT, bool VEC, typename SymIx>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(sizeof(SymIx) == 4 ? 8 : 1, 8)))
k_sym_part(const PartItem* __restrict__ items, const int* __restrict__ count_dev, int64_t annz,
           const int64_t* __restrict__ Acp, const int32_t* __restrict__ Air, const int64_t* __restrict__ Bcp,
           const int32_t* __restrict__ Bir, const int2* __restrict__ span, Split spl, int64_t* __restrict__ nnz,
           HeavyOut ho) {
  constexpr int T = 1 << (kPartLog - 5);   // bitmap words
  constexpr int WPT = T / NT;              // words per thread in the subwindow count (<= SUBW / 32)
  static_assert(WPT * 32 <= (1 << kSubLogMin), "a thread's words must lie in one subwindow");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  SymIx* qb = (SymIx*)smem;                        // NT
  SymIx* off = qb + NT;                            // NT
  int64_t* scr = (int64_t*)(off + NT);             // NT/64 + 1
  uint32_t* tab = (uint32_t*)(scr + NT / kWave + 1);// T
  int32_t* scnt = (int32_t*)(tab + T);             // part subwindows (<= 2^(kPartLog-kSubLogMin))
  int* misc = scnt + (1 << (kPartLog - kSubLogMin));   // [0] total
  int32_t* lens = misc + 8;                        // NT
  uint8_t* bvs = (uint8_t*)(lens + NT);            // NT
  const SegBuf<uint8_t, SymIx> sb{qb, off, bvs, scr, lens};
  const int count = *count_dev;
  // the segment [a0, a1) of B nonzero b (A column Bir[b]) inside part p0 (absolute part index) of the row space
  auto seg_in_part = [&](int32_t k, int32_t p0, int64_t& a0, int64_t& a1) {
    const int32_t pr0 = p0 << kPartLog;
    if (spl.ptab) {   // every A column narrowed to the part's rows: no gathers of rows outside it
      // one aligned row per column: its first entry's position, then the part offsets (one cache line, no Acp read)
      const int32_t* row = spl.ptab + (int64_t)k * spl.pstride;
      const int2 c = *(const int2*)row;
      const int64_t c0 = (int64_t)(uint32_t)c.x | ((int64_t)c.y << 32);
      a0 = c0 + row[2 + p0];
      a1 = c0 + row[3 + p0];
      return;
    }
    const int64_t c0 = Acp[k], c1 = Acp[k + 1];
    if (c1 - c0 >= kSplitMin) {
      const int32_t* t = spl.tab + (int64_t)spl.idx[k] * (spl.nsub + 1);
      a0 = c0 + t[pr0 >> spl.log];
      a1 = c0 + t[min(spl.nsub, (int32_t)(((int64_t)pr0 + (1 << kPartLog)) >> spl.log))];
    } else {
      a0 = c0;
      a1 = c1;
    }
  };
  int64_t cbase = 0, cleft = 0;   // thread 0: this workgroup's reserved rows (HeavyOut::chunk)
  STAMP_DECL
  STAMP(31);
  for (int i = blockIdx.x; i < count; i += gridDim.x) {
    const PartItem it = items[i];
    const int64_t bs = Bcp[it.j], be = Bcp[it.j + 1];
    const int2 sp = span[it.j];
    const int32_t r0 = ((sp.x >> kPartLog) + it.p) << kPartLog;
    const int32_t s0 = r0 >> spl.log;
    const int32_t s1 = min(spl.nsub, (int32_t)(((int64_t)r0 + (1 << kPartLog)) >> spl.log));
    for (int s = threadIdx.x; s < T; s += NT) tab[s] = 0;
    if (threadIdx.x < s1 - s0) scnt[threadIdx.x] = 0;
    if (threadIdx.x == 0) misc[0] = 0;
    __syncthreads();
    STAMP(26);
    auto seg = [&](int64_t b, int64_t& a0, int64_t& a1, uint8_t&) {
      seg_in_part(Bir[b], (sp.x >> kPartLog) + it.p, a0, a1);
    };
    auto ld = [&](int64_t q) { return Air[q]; };
    const RowLd4 ld4{Air, annz};
    auto ins = [&](int32_t r, uint8_t, int64_t, int64_t) {
      const uint32_t o = (uint32_t)(r - r0);
      if (o < (1u << kPartLog)) {
        const uint32_t bit = 1u << (o & 31);
#if CBG_SYM_TESTOR
        if (!(tab[o >> 5] & bit)) atomicOr(&tab[o >> 5], bit);
#else
        atomicOr(&tab[o >> 5], bit);
#endif
      }
    };
    if constexpr (VEC) for_each_multiply<NT, false, kUnrollSym, kGroupSym, uint8_t>(bs, be, sb, seg, ld4, ins);
    else for_each_multiply<NT, false, kUnrollSym, kGroupSym, uint8_t>(bs, be, sb, seg, ld, ins);
    __syncthreads();
    STAMP(27);
    int c = 0;
    uint32_t wds[WPT];
#pragma unroll
    for (int w = 0; w < WPT; ++w) {
      wds[w] = tab[threadIdx.x * WPT + w];
      c += __popc(wds[w]);
    }
    if (c) atomicAdd(&scnt[((r0 + threadIdx.x * WPT * 32) >> spl.log) - s0], c);
    int ptot;
    const int ex = block_excl_scan<NT>(c, lens, &ptot);   // lens is idle after the expansion
    if (threadIdx.x == 0) {
      misc[0] = ptot;
      int64_t off = -1;
      if (ho.rows && ptot > 0) {
        if (ho.chunk > 0) {   // rows from this workgroup's reservation: a global atomic every few parts, not every one
          // A part that does not fit the leftover gets its own exact reservation while the leftover is still >= chunk/8
          // (or the part is over half a chunk); a new chunk replaces a leftover < chunk/8, so at most 1/8 of a chunk is
          // dropped per chunk that was at least 7/8 used: waste <= used/7 + one chunk per workgroup (host sizing)
          if (ptot > cleft && (8 * cleft >= ho.chunk || 2 * (int64_t)ptot > ho.chunk)) {
            off = reserve_rows(ho, ptot);
          } else {
            if (ptot > cleft) {
              cbase = reserve_rows(ho, ho.chunk);
              cleft = cbase >= 0 ? ho.chunk : 0;
            }
            if (ptot <= cleft) {
              off = cbase;
              cbase += ptot;
              cleft -= ptot;
            }
          }
        } else {
          off = reserve_rows(ho, ptot);
        }
        ho.poff[(int64_t)it.h * kMaxParts + it.p] = off;
        atomicOr(&ho.mode[it.h], off >= 0 ? 2 : 16);
      }
      misc[4] = (int)(off & 0xffffffff);
      misc[5] = (int)(off >> 32);
    }
    __syncthreads();
    STAMP(28);
    const int64_t off = (int64_t)(uint32_t)misc[4] | ((int64_t)misc[5] << 32);
    const int ptot_u = misc[0];
    if (CBG_SYM_ROWS_LDS && off >= 0 && ptot_u <= T) {
      // the bitmap is in registers (wds): its LDS holds the part's rows in order, then the workgroup copies them out
      // with consecutive lanes on consecutive rows (whole cache lines per store instruction)
      int pos = ex;
#pragma unroll
      for (int w = 0; w < WPT; ++w) {
        uint32_t wd = wds[w];
        while (wd) {
          const int b = __ffs(wd) - 1;
          wd &= wd - 1;
          tab[pos++] = (uint32_t)(r0 + 32 * (threadIdx.x * WPT + w) + b);
        }
      }
      __syncthreads();
      for (int x = threadIdx.x; x < ptot_u; x += NT) ho.rows[off + x] = (HRow)tab[x];
    } else if (off >= 0) {   // this part's sorted rows for the numeric pass (each thread: its words' rows)
      int64_t pos = off + ex;
#pragma unroll
      for (int w = 0; w < WPT; ++w) {
        uint32_t wd = wds[w];
        while (wd) {
          const int b = __ffs(wd) - 1;
          wd &= wd - 1;
          ho.rows[pos++] = (HRow)(r0 + 32 * (threadIdx.x * WPT + w) + b);
        }
      }
    }
    if (threadIdx.x == 0 && misc[0]) atomicAdd((unsigned long long*)&nnz[it.j], (unsigned long long)misc[0]);
    const int32_t sf = max(s0, sp.x >> spl.log), sl = min(s1 - 1, sp.y >> spl.log);
    int32_t* dst = ho.sub + (int64_t)it.h * ho.nsub;
    for (int s = sf + (int)threadIdx.x; s <= sl; s += NT) dst[s] = scnt[s - s0];
    __syncthreads();
    STAMP(29);
    STAMP_COUNT(30, 1);
  }
}

// Part table of A for k_sym_part: for every A column the entry offsets of the 2^kPartLog-row part boundaries (P + 1 per
// column), so a part's item gathers only the rows inside the part -- without it a short column (no split-table row) is
// read whole by every part of every wide column it feeds (8 parts at 2^21 rows).  One thread per column: a linear walk
// over a short column's sorted rows, binary searches in a long one.  Row k = [Acp[k] (two words), offsets 0..P], PS
// words (a power of two >= P + 3), so a part's lookup reads one cache line and no column pointer.
__global__ void __launch_bounds__(256) k_part_table(int64_t ncol, const int64_t* __restrict__ Acp,
                                                    const int32_t* __restrict__ Air, int32_t P, int32_t PS,
                                                    int32_t* __restrict__ ptab) {
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < ncol; k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c0 = Acp[k], c1 = Acp[k + 1];
    int32_t* row = ptab + k * PS;
    *(int2*)row = make_int2((int32_t)(uint32_t)(c0 & 0xffffffff), (int32_t)(c0 >> 32));
    int32_t* t = row + 2;
    t[0] = 0;
    if (c1 - c0 <= 64) {
      int64_t i = c0;
      for (int p = 1; p < P; ++p) {
        const int64_t lim = (int64_t)p << kPartLog;
        while (i < c1 && Air[i] < lim) ++i;
        t[p] = (int32_t)(i - c0);
      }
    } else {
      int64_t i = c0;
      for (int p = 1; p < P; ++p) {
        i = lower_bound_rows(Air, i, c1, (int64_t)p << kPartLog);
        t[p] = (int32_t)(i - c0);
      }
    }
    t[P] = (int32_t)(c1 - c0);
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

// ============================================================================ 5. heavy-column units
// one wavefront per long column: every subwindow boundary by binary search
__global__ void __launch_bounds__(256) k_split_fill(int nlong, const int32_t* __restrict__ longcols,
                                                    const int64_t* __restrict__ Acp, const int32_t* __restrict__ Air,
                                                    int32_t* __restrict__ tab, int32_t nsub, int32_t log) {
  const int w = threadIdx.x / kWave, l = lane_id();
  for (int64_t e = blockIdx.x * 4 + w; e < nlong; e += (int64_t)gridDim.x * 4) {
    const int32_t k = longcols[e];
    const int64_t c0 = Acp[k], c1 = Acp[k + 1];
    int32_t* t = tab + e * (nsub + 1);
    for (int s = l; s <= nsub; s += kWave) t[s] = (int32_t)(lower_bound_rows(Air, c0, c1, (int64_t)s << log) - c0);
  }
}
// Unit caps per semiring.  Rank mode (k_num_heavy) needs cnt*sizeof(Acc) value slots plus a
// span/32-word bitmap inside the (T+NT)*(sizeof(Acc)+4)-byte vals+keys region, and at most 2T
// bitmap words (one 16-bit directory entry per word pair): span <= 8*((T+NT)*(sA+4) - cap*sA).
// A semiring without rank mode (BoolCopy: its hash detects a second contribution) caps units at T/2
// outputs so the order-preserving hash keeps load <= 1/2.
template <class SRT>
constexpr int64_t heavy_unit_cap() {
  return SRT::kAddIsError || !CBG_RANK_MODE ? (int64_t)(1 << CBG_HEAVY_LOGT) / 2 : kUnitCap;
}
// Round 6: a unit's span also grows with the LDS its values leave free -- a unit of cnt outputs fits the rows-known
// kernel while cnt*sA (padded) + 4*(span/32 + 2) <= (T+NT)*(sA+4) and span <= 64T (the pair-word directory) -- so a
// sparse, span-limited unit takes up to 64T rows instead of the cap a full unit needs: s20 heavy 29.6 -> 27.6 ms, s21
// 201.8 -> 194.3 ms per product, s22 2x2x2 rank 0 83.7 -> 80.7 ms (same-box A/B, profiles/r06l_span_adaptive_ab.txt)
template <class SRT>
constexpr int64_t heavy_rank_bytes() {   // 0: no rank mode (the fixed span cap alone)
  constexpr int64_t T = 1 << CBG_HEAVY_LOGT, NT = CBG_HEAVY_NT, sA = sizeof(typename SRT::Acc);
  return SRT::kAddIsError || !CBG_RANK_MODE ? 0 : (T + NT) * (sA + 4);
}
template <class SRT>
constexpr int64_t heavy_span_cap() {
  constexpr int64_t T = 1 << CBG_HEAVY_LOGT, NT = CBG_HEAVY_NT, sA = sizeof(typename SRT::Acc);
  constexpr int64_t fit = 8 * ((T + NT) * (sA + 4) - kUnitCap * sA);
  constexpr int64_t dir = 64 * T;
  constexpr int64_t cap = fit < dir ? fit : dir;
  if (SRT::kAddIsError || !CBG_RANK_MODE || CBG_RANK_SPAN_CAP <= 0) return 0;
  return CBG_RANK_SPAN_CAP < cap ? CBG_RANK_SPAN_CAP : cap;
}

// what the heavy kernels process (columns with nnz > kHeavy): multiplies, B nonzeros and outputs, summed into
// out[0..2] -- the per-unit figures of SURVEY 8(d)'s algorithmic bytes of the dominant kernels (cbg_profile)
__global__ void __launch_bounds__(256) k_heavy_sums(int H, const int32_t* __restrict__ cols,
                                                    const int64_t* __restrict__ flop, const int64_t* __restrict__ nnz,
                                                    const int64_t* __restrict__ Bcp, unsigned long long* __restrict__ out) {
  int64_t f = 0, b = 0, c = 0;
  for (int h = blockIdx.x * blockDim.x + threadIdx.x; h < H; h += gridDim.x * blockDim.x) {
    const int32_t j = cols[h];
    const int64_t z = nnz[j];
    if (z > kHeavy) {
      f += flop[j];
      b += Bcp[j + 1] - Bcp[j];
      c += z;
    }
  }
  f = wave_sum64(f);
  b = wave_sum64(b);
  c = wave_sum64(c);
  if (lane_id() == 0 && (f | b | c)) {
    atomicAdd(out + 0, (unsigned long long)f);
    atomicAdd(out + 1, (unsigned long long)b);
    atomicAdd(out + 2, (unsigned long long)c);
  }
}

// units of a heavy column: consecutive subwindows while the running count stays <= unit_cap
// unit_cap / span_cap come from the semiring (heavy_unit_caps): rank-mode accumulators hold up to
// kUnitCap outputs over a bounded span; hash-only semirings (BoolCopy) keep load <= 1/2.
// One thread per column walks its subwindow counts in chunks of kBuildChunk, loaded together into the thread's LDS
// slice (one load latency per chunk instead of one per subwindow).
constexpr int kBuildChunk = 16;
__global__ void __launch_bounds__(256) k_build_units(int H, const int32_t* __restrict__ cols, const int32_t* __restrict__ sub, int32_t nsub,
                              int32_t log, int64_t unit_cap, int64_t span_cap, int64_t rank_bytes, int32_t acc_bytes,
                              const int2* __restrict__ span, const int64_t* __restrict__ colptr,
                              const int64_t* __restrict__ Bcp, Unit* __restrict__ units, int64_t* __restrict__ ucnt,
                              int2* __restrict__ uspan, int64_t* __restrict__ nnz, int32_t* __restrict__ nunits,
                              int64_t* __restrict__ segsz, int64_t* __restrict__ icnt,
                              const int32_t* __restrict__ hmode, const int64_t* __restrict__ hpoff,
                              UnitRows* __restrict__ urows) {
  const int h = blockIdx.x * blockDim.x + threadIdx.x;
  if (h >= H) return;
  const int32_t j = cols[h];
  if (nnz[j] <= kHeavy) {   // a wide column (registered before its count was known) that stayed light
    nunits[h] = 0;
    segsz[h] = 0;
    icnt[h] = 0;
    return;
  }
  const int2 sp = span[j];
  const int32_t sf = sp.x >> log, sl = sp.y >> log;
  const int32_t* c = sub + (int64_t)h * nsub;
  const int64_t slot = (int64_t)h * nsub;
  int64_t out = colptr[j];
  int u = 0, st = sf;
  int64_t acc = 0;
  // where each subwindow's rows lie in the symbolic row scratch (mode 1: one run for the column,
  // mode 2: one run per 2^kPartLog-row part, parts relative to the column's first part)
  const int32_t mode = hmode ? hmode[h] : 0;
  const int pshift = kPartLog - log;   // subwindows -> parts
  const int32_t P0 = sp.x >> kPartLog;
  int64_t pfx_col = 0, pfx_part = 0;
  int32_t curP = -1;
  UnitRows ur{};
  int64_t poff_cur = -1, pn_cur = 0;
  auto close_piece = [&]() {
    if (pn_cur > 0) {
      if (ur.np < 3) { ur.off[ur.np] = poff_cur; ur.n[ur.np] = (int32_t)pn_cur; ++ur.np; }
      else ur.np = 4;   // cannot happen (span cap < 2 parts): rows unknown for this unit
    }
    pn_cur = 0;
    poff_cur = -1;
  };
  auto emit = [&](int32_t s0, int32_t s1, int64_t n) {
    units[slot + u] = Unit{j, s0, s1, (int32_t)n, out, -1};
    ucnt[slot + u] = n;
    const int64_t lo = max((int64_t)sp.x, (int64_t)s0 << log);
    const int64_t hi = min((int64_t)sp.y, ((int64_t)s1 << log) - 1);
    uspan[slot + u] = make_int2((int32_t)lo, (int32_t)hi);
    close_piece();
    if (mode != 1 && mode != 2) ur.np = 0;
    if (ur.np > 3) ur.np = 0;
    if (urows) urows[slot + u] = ur;
    ur = UnitRows{};
    ++u;
    out += n;
  };
  __shared__ int32_t cs[256 * (kBuildChunk + 1)];   // odd stride: the lanes' slices start in distinct banks
  int32_t* my = cs + threadIdx.x * (kBuildChunk + 1);
  for (int32_t s = sf; s <= sl; ++s) {
    if (((s - sf) & (kBuildChunk - 1)) == 0) {
      int32_t r[kBuildChunk];
#pragma unroll
      for (int q = 0; q < kBuildChunk; ++q) r[q] = s + q <= sl ? c[s + q] : 0;
#pragma unroll
      for (int q = 0; q < kBuildChunk; ++q) my[q] = r[q];
    }
    const int64_t n = my[(s - sf) & (kBuildChunk - 1)];
    if (acc == 0) st = s;   // a unit starts at its first non-empty subwindow (empty gaps span nothing)
    const int64_t sub_span = (int64_t)(s + 1 - st) << log;
    int64_t cap = span_cap;
    if (rank_bytes > 0) {   // adaptive: the LDS the unit's values leave to its bitmap, within the directory's 64T rows
      const int64_t cpad = (acc + n + 1) & ~(int64_t)1;
      cap = min((int64_t)64 << CBG_HEAVY_LOGT, 8 * (rank_bytes - cpad * acc_bytes - 8));
    }
    const bool wide = span_cap > 0 && sub_span > cap;
    if (acc > 0 && (acc + n > unit_cap || wide)) {
      emit(st, s, acc);
      st = s;
      acc = 0;
    }
    // this subwindow's rows in the scratch
    int64_t ro = -1;
    if (mode == 1) {
      ro = hpoff[(int64_t)h * kMaxParts] + pfx_col;
    } else if (mode == 2) {
      const int32_t P = s >> pshift;
      if (P != curP) { curP = P; pfx_part = 0; }
      const int32_t pr = P - P0;
      ro = (pr >= 0 && pr < kMaxParts) ? hpoff[(int64_t)h * kMaxParts + pr] + pfx_part : -1;
    }
    if (n > 0) {
      if (pn_cur > 0 && ro == poff_cur + pn_cur) pn_cur += n;
      else { close_piece(); poff_cur = ro; pn_cur = n; }
    }
    acc += n;
    pfx_col += n;
    pfx_part += n;
  }
  if (acc > 0) emit(st, sl + 1, acc);
  nnz[j] = 0;   // the whole column is now covered by units
  nunits[h] = u;
  segsz[h] = (int64_t)u * (Bcp[j + 1] - Bcp[j]);
  icnt[h] = (u + kItemUnits - 1) / kItemUnits;
}

// Segment table of every unit: for each heavy column, each B nonzero b = (k, B(k,j)) is visited once and its A column's
// boundaries for all of the column's units are written (split-table entries, mostly from cache, instead of a dependent
// lookup chain per (unit, b) inside the numeric kernel).  Short A columns are given whole (rows outside a unit are
// dropped at insert time) unless their row range misses the unit entirely.  The column's unit bounds are staged in LDS
// and four units' split-table entries are loaded at once; a column with fewer B nonzeros than the workgroup's lanes
// spreads its units over lane groups (~80 B nonzeros per heavy column).  Against one lane per B nonzero walking its
// units with a scalar load each: s20 63.8 -> 63.6 ms, s22 rank panel 80.6 -> 79.9 ms (profiles/r06s_unit_segs_ab.txt).
template <class SRT, int LOGT, int NT>
__global__ void __launch_bounds__(256) k_unit_segs(const int32_t* __restrict__ cols, const int32_t* __restrict__ nunits,
                                                       const int64_t* __restrict__ segoff, Unit* __restrict__ units,
                                                       int32_t nsub, const int64_t* __restrict__ Acp,
                                                       const int4* __restrict__ ainfo, const int64_t* __restrict__ Bcp,
                                                       const int32_t* __restrict__ Bir, Split sp, UnitSeg* __restrict__ seg) {
  __shared__ int2 us[kMaxSub];
  const int h = blockIdx.x;
  const int nu = nunits[h];
  if (nu == 0) return;   // uniform
  const int32_t j = cols[h];
  const int64_t bs = Bcp[j], nb = Bcp[j + 1] - bs;
  const int64_t base = segoff[h];
  Unit* U = units + (int64_t)h * nsub;
  for (int u = threadIdx.x; u < nu; u += blockDim.x) {
    U[u].segbase = base + (int64_t)u * nb;
    us[u] = make_int2(U[u].s0, U[u].s1);
  }
  __syncthreads();
  // lane groups: G groups of nb lanes when nb < 256 (group g takes units g, g+G, ...), else one group striding over nb
  const int G = nb < (int64_t)blockDim.x ? (int)(blockDim.x / nb) : 1;
  const int g = nb < (int64_t)blockDim.x ? (int)(threadIdx.x / nb) : 0;
  if (g >= G) return;
  const int64_t istep = nb < (int64_t)blockDim.x ? nb : (int64_t)blockDim.x;
  for (int64_t i = nb < (int64_t)blockDim.x ? (int64_t)threadIdx.x % nb : threadIdx.x; i < nb; i += istep) {
    const int32_t k = Bir[bs + i];
    const int64_t c0 = Acp[k];
    const int4 ai = ainfo[k];   // (length, first row, last row, split-table row)
    const int64_t c1 = c0 + ai.x;
    UnitSeg* out = seg + base + i;
    if (ai.w >= 0) {
      const int32_t* t = sp.tab + (int64_t)ai.w * (sp.nsub + 1);
      for (int u = g; u < nu; u += 4 * G) {
        int32_t lo[4], hi[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {   // four units' entries in flight together
          const int2 b2 = us[min(u + q * G, nu - 1)];
          lo[q] = t[b2.x];
          hi[q] = t[b2.y];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (u + q * G < nu) out[(int64_t)(u + q * G) * nb] = UnitSeg{c0 + lo[q], c0 + hi[q]};
      }
    } else {
      // a short column: whole, when its first..last rows overlap the unit (the sweep drops the other rows).
      // Narrowing it by binary search was measured: k_unit_segs 2.5 -> 5.1 ms for 0.6 ms of heavy sweep (r03r)
      const int32_t rf = ai.y, rl = ai.z;   // (INT32_MAX, -1) for an empty column: never hits
      for (int u = g; u < nu; u += G) {
        const int2 b2 = us[u];
        const bool hit = c1 > c0 && rl >= ((int64_t)b2.x << sp.log) && rf < ((int64_t)b2.y << sp.log);
        out[(int64_t)u * nb] = hit ? UnitSeg{c0, c1} : UnitSeg{c0, c0};
      }
    }
  }
}
// overflowed (hash) units -> single-subwindow units, which run in dense mode
__global__ void k_split_overflow_units(const int* __restrict__ n_ovf, const int32_t* __restrict__ ovf,
                                       const Unit* __restrict__ units, const int32_t* __restrict__ sub, int32_t nsub,
                                       Unit* __restrict__ out_units,
                                       int* __restrict__ n_out, int32_t* __restrict__ out_list) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= *n_ovf) return;
  const int32_t uid = ovf[i];
  const Unit u = units[uid];
  const int64_t h = uid / nsub;   // units of heavy column h live at [h*nsub, (h+1)*nsub)
  int64_t off = u.outoff;
  for (int32_t s = u.s0; s < u.s1; ++s) {
    const int32_t n = sub[h * nsub + s];
    if (n > 0) {
      const int e = atomicAdd(n_out, 1);
      out_units[e] = Unit{u.j, s, s + 1, n, off, -1};
      out_list[e] = e;
      off += n;
    }
  }
}

// ============================================================================ 6. numeric
// Output: C.row / C.val at colptr[j] .. colptr[j+1], rows ascending.
template <typename V>
struct NumOut {
  int32_t* row;
  V* val;
  int* adderr;            // BoolCopy add() attempted
  int* ovf_n;             // fallback list length
  int32_t* ovf_list;      // items whose order-preserving hash overflowed (columns, or unit ids)
};

// numeric pass of the one-lane columns (kLaneClass / kLane8Class, see k_sym_lane): LMAX table entries per lane
// (its LDS slice bounds the lanes a CU holds: 16 -> 3 workgroups of 256 per CU for f64, 8 -> 5)
template <class SRT, typename V, int LMAX>
__global__ void __launch_bounds__(256) k_num_lane(const int32_t* __restrict__ list, int64_t count, DevCsc<V> A,
                                                  DevCsc<V> B, const int64_t* __restrict__ colptr, NumOut<V> out) {
  using Acc = typename SRT::Acc;
  constexpr int STRIDE = LMAX + 1;   // odd stride: the 64 lanes' slices start in distinct banks
  __shared__ int32_t s_rows[256 * STRIDE];
  __shared__ Acc s_acc[256 * STRIDE];
  int32_t* rows = s_rows + threadIdx.x * STRIDE;
  Acc* accs = s_acc + threadIdx.x * STRIDE;
  bool aerr = false;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < count; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t j = list[i];
    int m = 0;
    const int64_t bs = B.cp[j], be = B.cp[j + 1];
    auto insert = [&](int32_t r, const Acc& x) {
      int y = 0;
      while (y < m && rows[y] != r) ++y;
      if (y == m) {
        if (m == LMAX) return;   // cannot happen: flop <= LMAX
        rows[m] = r;
        accs[m] = SRT::identity();
        ++m;
      } else if (SRT::kAddIsError) {
        aerr = true;
      }
      SRT::acc(&accs[y], x);
    };
    // (B nonzero, A entry) in storage order: the first contributor of a row is the first inserted.  The B
    // nonzeros go kLaneBatch at a time: their rows, A ranges and the first A entry of every range are loaded
    // with independent loads before the inserts (a serial B -> A.cp -> A.ir chain per nonzero otherwise)
    for (int64_t b0 = bs; b0 < be; b0 += kLaneBatch) {
      int32_t k[kLaneBatch];
      int64_t a0[kLaneBatch], a1[kLaneBatch];
      int32_t r0[kLaneBatch];
      V av0[kLaneBatch], bv[kLaneBatch];
#pragma unroll
      for (int t = 0; t < kLaneBatch; ++t) k[t] = b0 + t < be ? B.ir[b0 + t] : 0;
#pragma unroll
      for (int t = 0; t < kLaneBatch; ++t) {
        const bool ok = b0 + t < be;
        a0[t] = ok ? A.cp[k[t]] : 0;
        a1[t] = ok ? A.cp[k[t] + 1] : 0;
        bv[t] = ok ? load_val(B.val, b0 + t) : V(0);
      }
#pragma unroll
      for (int t = 0; t < kLaneBatch; ++t) {
        const bool ok = a1[t] > a0[t];
        r0[t] = ok ? A.ir[a0[t]] : 0;
        av0[t] = ok ? load_val(A.val, a0[t]) : V(0);
      }
#pragma unroll
      for (int t = 0; t < kLaneBatch; ++t) {
        if (a1[t] <= a0[t]) continue;
        const int64_t b = b0 + t;
        insert(r0[t], SRT::mul(av0[t], bv[t], a0[t], b));
        for (int64_t q = a0[t] + 1; q < a1[t]; ++q) insert(A.ir[q], SRT::mul(load_val(A.val, q), bv[t], q, b));
      }
    }
    for (int x = 1; x < m; ++x) {   // insertion sort by row (m <= kLaneMax)
      const int32_t r = rows[x];
      const Acc v = accs[x];
      int y = x - 1;
      while (y >= 0 && rows[y] > r) {
        rows[y + 1] = rows[y];
        accs[y + 1] = accs[y];
        --y;
      }
      rows[y + 1] = r;
      accs[y + 1] = v;
    }
    const int64_t o = colptr[j];
    for (int x = 0; x < m; ++x) {
      out.row[o + x] = rows[x];
      out.val[o + x] = SRT::out(accs[x], A.val, B.val);
    }
  }
  if (aerr) atomicOr(out.adderr, 1);
}


template <bool UNIT>
__device__ __forceinline__ Work get_work(const int32_t* __restrict__ list, int64_t i, const Unit* __restrict__ units,
                                         const int2* __restrict__ span, const int64_t* __restrict__ colptr,
                                         int32_t log) {
  Work w;
  if constexpr (UNIT) {
    const Unit u = units[list[i]];
    const int2 sp = span[u.j];
    w.j = u.j;
    w.s0 = u.s0;
    w.s1 = u.s1;
    w.lo = (int32_t)max((int64_t)sp.x, (int64_t)u.s0 << log);
    w.hi = (int32_t)min((int64_t)sp.y, ((int64_t)u.s1 << log) - 1);
    w.ob = u.outoff;
    w.segbase = u.segbase;
  } else {
    const int32_t j = list[i];
    const int2 sp = span[j];
    w.j = j;
    w.s0 = w.s1 = -1;
    w.lo = sp.x;
    w.hi = sp.y;
    w.ob = colptr ? colptr[j] : 0;
    w.segbase = -1;
  }
  return w;
}

template <typename V>
struct NumItem {
  int32_t r;
  V a;
};

// (row, value) loader with a paired path: expand_staged_slots loads a lane's group of 2 consecutive A entries as
// one 8-byte row load and one 2*sizeof(V) value load (CBG_NUM_VEC2, default on) instead of two of each.  At the
// end of A the pair is moved back to stay in bounds (the entry past the segment is never accumulated).
#ifndef CBG_NUM_VEC2
#define CBG_NUM_VEC2 1
#endif
template <typename V, bool AV>
struct NumLd2 {
  const int32_t* ir;
  const V* val;
  int64_t n;   // entries of A (>= 2 for the paired path)
  __device__ __forceinline__ NumItem<V> operator()(int64_t q) const { return NumItem<V>{ir[q], AV ? val[q] : V(1)}; }
  __device__ __forceinline__ void vec2(int64_t q, NumItem<V>& x, NumItem<V>& y) const {
    const int64_t qv = q + 2 <= n ? q : n - 2;
    int32_t r[2];
    V v[2] = {V(1), V(1)};
    __builtin_memcpy(r, ir + qv, 8);
    if (AV) __builtin_memcpy(v, val + qv, 2 * sizeof(V));
    if (q != qv) { r[0] = r[1]; v[0] = v[1]; }
    x = NumItem<V>{r[0], v[0]};
    y = NumItem<V>{r[1], v[1]};
  }
};
template <typename V, bool AV> struct HasVec2<NumLd2<V, AV>> { static constexpr bool value = true; };

// Compaction of an order-preserving hash table of Tcap slots by NT lanes.
// out position of an occupied slot s = (#occupied before its run start) + (#keys in its run smaller).
template <class SRT, typename V>
__device__ __forceinline__ void compact_hash_runs(const int32_t* keys, const typename SRT::Acc* vals, int Tcap,
                                                  int occ_before_chunk, int c0, int c1, int64_t outbase,
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

// Block compaction of an order-preserving hash table (TC = Te + NT slots, CH = TC/NT <= CHMAX per
// thread) into C(:, ...) at `ob`: run-rank positions are computed from the table into registers,
// the table is then reused as a staging buffer in output order, and the staged block is written
// with consecutive lanes on consecutive addresses (coalesced) instead of one scattered store per
// entry.  Contains barriers; the caller synchronises before the table is re-initialised.
// Block compaction of an order-preserving hash table into C(:, ...) at `ob`, sorted by row, with no
// per-run scans (a run-walking compaction is SIMD-divergent: a wave pays for the longest run among
// its lanes).  home(r) is monotone in r, so the keys with a smaller home all precede r: with
// cnt[h] = #keys whose home is h, r's output position is excl_scan(cnt)[home(r)] plus its rank among
// the (rare, tiny) group of keys sharing its home.
//   1. cnt[h] in LDS as packed 16-bit halves (hc: Te/2 words, caller-provided scratch);
//   2. exclusive scan of the Te counts in place;
//   3. each key takes base[h] + an atomic cursor, kept in registers with its accumulator;
//   4. the table is reused as the staging buffer: (row, acc) written at their positions, then every
//      home group of >= 2 keys is insertion-sorted by the thread owning that home;
//   5. the staged block is written out coalesced.
// TC = table slots (Te + tail), CH = ceil(TC/NT) <= CHMAX slots per thread (contiguous chunks).
// hc (Te/2 words) must be zero on entry (the caller clears it with the table).
// Contains barriers; the caller synchronises before the table is re-initialised.
template <class SRT, typename V, int NT, int CHMAX>
__device__ __forceinline__ void compact_hash_homes(int32_t* keys, typename SRT::Acc* vals, int TC, int Te,
                                                   int32_t lo, uint32_t mult, uint32_t* hc, int* scan,
                                                   int64_t ob, const V* aval, const V* bval, int32_t* orow,
                                                   V* oval) {
  using Acc = typename SRT::Acc;
  const int CH = (TC + NT - 1) / NT;
  const int c0 = threadIdx.x * CH;
  const int NW = Te >> 1;                        // packed count words
  STAMP_DECL
  STAMP(14);
  // 1. count keys per home; the returned count is the key's index inside its home group
  int32_t rk[CHMAX];
  Acc rv[CHMAX];
  uint32_t hm[CHMAX];
  int ix[CHMAX];
#pragma unroll
  for (int i = 0; i < CHMAX; ++i) {
    const int sl = c0 + i;
    rk[i] = (i < CH && sl < TC) ? keys[sl] : kEmpty;
    hm[i] = 0;
    ix[i] = 0;
    if (rk[i] != kEmpty) {
      hm[i] = mono_home(rk[i], lo, mult);
      rv[i] = vals[sl];
      const uint32_t sh = 16 * (hm[i] & 1);
      ix[i] = (int)((atomicAdd(&hc[hm[i] >> 1], 1u << sh) >> sh) & 0xffffu);
    }
  }
  __syncthreads();
  STAMP(15);
  // 2. exclusive scan over the Te 16-bit counts in place: hc half h = base(h)
  const int WP = (NW + NT - 1) / NT;
  const int w0 = min(NW, (int)threadIdx.x * WP), w1 = min(NW, w0 + WP);
  int local = 0;
  for (int w = w0; w < w1; ++w) {
    const uint32_t x = hc[w];
    local += (int)(x & 0xffffu) + (int)(x >> 16);
  }
  int tot;
  int run = block_excl_scan<NT>(local, scan, &tot);
  for (int w = w0; w < w1; ++w) {
    const uint32_t x = hc[w];
    const uint32_t c_lo = x & 0xffffu, c_hi = x >> 16;
    hc[w] = (uint32_t)run | ((uint32_t)(run + (int)c_lo) << 16);
    run += (int)(c_lo + c_hi);
  }
  __syncthreads();
  STAMP(16);
  // 3. positions: group base + index inside the group
  int ro[CHMAX];
#pragma unroll
  for (int i = 0; i < CHMAX; ++i) {
    ro[i] = -1;
    if (rk[i] != kEmpty) {
      const uint32_t h = hm[i];
      ro[i] = (int)((hc[h >> 1] >> (16 * (h & 1))) & 0xffffu) + ix[i];
    }
  }
  __syncthreads();   // every table read is done: reuse keys/vals as the staging buffer
  STAMP(17);
#pragma unroll
  for (int i = 0; i < CHMAX; ++i)
    if (ro[i] >= 0) {
      keys[ro[i]] = rk[i];
      vals[ro[i]] = rv[i];
    }
  __syncthreads();
  STAMP(18);
  // 4. keys sharing a home (1-3 at load <= 0.5) were staged contiguously but in arbitrary order:
  //    every output position computes its key's rank inside its group with independent reads of the
  //    group (no dependent chains), then all keys move after one barrier
  constexpr int PMAX = CHMAX;                    // tot <= Te/2 <= CHMAX * NT
  int pp[PMAX];
  int32_t pk[PMAX];
  Acc pv[PMAX];
#pragma unroll
  for (int i = 0; i < PMAX; ++i) {
    const int p = (int)threadIdx.x + i * NT;
    pp[i] = -1;
    if (p < tot) {
      const int32_t k = keys[p];
      const uint32_t h = mono_home(k, lo, mult);
      const int st = (int)((hc[h >> 1] >> (16 * (h & 1))) & 0xffffu);
      const int en = (h + 1 < (uint32_t)Te) ? (int)((hc[(h + 1) >> 1] >> (16 * ((h + 1) & 1))) & 0xffffu) : tot;
      int r = 0;
      for (int q = st; q < en; ++q) r += (keys[q] < k);
      pp[i] = st + r;
      pk[i] = k;
      pv[i] = vals[p];
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < PMAX; ++i)
    if (pp[i] >= 0) {
      keys[pp[i]] = pk[i];
      vals[pp[i]] = pv[i];
    }
  __syncthreads();
  STAMP(19);
  for (int i = threadIdx.x; i < tot; i += NT) {
    orow[ob + i] = keys[i];
    oval[ob + i] = SRT::out(vals[i], aval, bval);
  }
  STAMP(20);
}

// ---- wave numeric: one item per wavefront, table T slots (+kTail) per wave
constexpr int kTail = 64;

// one numeric insert (dense: bitmap + value slot; hash: order-preserving open addressing).  Unit
// items drop rows outside their range (whole short A columns, see unit_bounds).
template <class SRT, typename V, bool UNIT>
__device__ __forceinline__ void num_insert(Table<typename SRT::Acc>& t, bool dense, const Work& wk, uint32_t mult,
                                           const NumItem<V>& it, V bv, int64_t q, int64_t b, int& ovf, int& aerr) {
  using Acc = typename SRT::Acc;
  if constexpr (UNIT)
    if (it.r < wk.lo || it.r > wk.hi) return;
  const Acc x = SRT::mul(it.a, bv, q, b);
  if (dense) {
    const int32_t o = it.r - wk.lo;
    const uint32_t bit = 1u << (o & 31);
    const uint32_t old = atomicOr((uint32_t*)&t.keys[o >> 5], bit);
    if (SRT::kAddIsError && (old & bit)) aerr = 1;
    SRT::acc(&t.vals[o], x);
  } else {
    if (!hash_insert_num<SRT>(t, it.r, mono_home(it.r, wk.lo, mult), x, &aerr)) ovf = 1;
  }
}

template <typename V, bool UNIT>
__device__ __forceinline__ void num_seg(const DevCsc<V>& A, const DevCsc<V>& B, const Split& spl,
                                        const UnitSeg* __restrict__ useg, const Work& wk, int64_t b, int64_t& a0,
                                        int64_t& a1, V& bv) {
  if constexpr (UNIT) {
    if (wk.segbase >= 0) {
      const UnitSeg sg = useg[wk.segbase + (b - B.cp[wk.j])];
      a0 = sg.a0;
      a1 = sg.a1;
    } else {
      unit_bounds(A.cp, spl, B.ir[b], wk.s0, wk.s1, a0, a1);
    }
  } else {
    const int32_t k = B.ir[b];
    a0 = A.cp[k];
    a1 = A.cp[k + 1];
  }
  bv = load_val(B.val, b);
}

template <class SRT, typename V, int LOGT, bool UNIT>
__global__ void __launch_bounds__(256) k_num_wave(const int32_t* __restrict__ list, int64_t count,
                                                  const Unit* __restrict__ units, DevCsc<V> A, DevCsc<V> B,
                                                  const int2* __restrict__ span, const int64_t* __restrict__ colptr,
                                                  Split spl, NumOut<V> out) {
  using Acc = typename SRT::Acc;
  constexpr int T = 1 << LOGT;
  constexpr int TC = T + kTail;
  __shared__ int32_t s_keys[4][TC];
  __shared__ Acc s_vals[4][TC];
  __shared__ int64_t s_qb[4][kWave], s_off[4][kWave];
  __shared__ V s_bv[4][kWave];
  __shared__ int32_t s_len[4][kWave];
  const int w = threadIdx.x / kWave, l = lane_id();
  Table<Acc> t{s_keys[w], s_vals[w], T, TC};
  const SegBuf<V> sb{s_qb[w], s_off[w], s_bv[w], nullptr, s_len[w]};
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  for (int64_t i = blockIdx.x * 4 + w; i < count; i += nwaves) {
    const Work wk = get_work<UNIT>(list, i, units, span, colptr, spl.log);
    const int64_t spn = (int64_t)wk.hi - wk.lo + 1;
    const bool dense = spn <= T;
    const uint32_t mult = dense ? 0u : (uint32_t)(((uint64_t)T << 32) / (uint64_t)spn);
    for (int s = l; s < TC; s += kWave) { t.keys[s] = dense ? 0 : kEmpty; t.vals[s] = SRT::identity(); }
    wave_sync();
    int ovf = 0, aerr = 0;
    for_each_multiply<kWave, true, kUnroll, kGroupNum, V>(
        B.cp[wk.j], B.cp[wk.j + 1], sb,
        [&](int64_t b, int64_t& a0, int64_t& a1, V& bv) { num_seg<V, UNIT>(A, B, spl, spl.useg, wk, b, a0, a1, bv); },
        [&](int64_t q) { return NumItem<V>{A.ir[q], load_val(A.val, q)}; },
        [&](const NumItem<V>& it, V bv, int64_t q, int64_t b) {
          num_insert<SRT, V, UNIT>(t, dense, wk, mult, it, bv, q, b, ovf, aerr);
        });
    wave_sync();
    const bool wov = __any(ovf);
    if (__any(aerr) && l == 0) atomicOr(out.adderr, 1);
    const int64_t ob = wk.ob;
    if (wov) {
      if (l == 0) out.ovf_list[atomicAdd(out.ovf_n, 1)] = list[i];
    } else if (dense) {
      constexpr int NWORD = T / 32;   // <= 16 for T <= 512
      uint32_t wd = (l < NWORD) ? (uint32_t)t.keys[l] : 0u;
      const int pc = __popc(wd);
      int o = wave_incl_scan(pc) - pc;
      while (wd) {
        const int bpos = __ffs(wd) - 1;
        wd &= wd - 1;
        const int rr = l * 32 + bpos;
        out.row[ob + o] = wk.lo + rr;
        out.val[ob + o] = SRT::out(t.vals[rr], A.val, B.val);
        ++o;
      }
    } else {
      constexpr int CH = TC / kWave;
      const int c0 = l * CH, c1 = c0 + CH;
      int occ = 0;
      for (int s = c0; s < c1; ++s) occ += (t.keys[s] != kEmpty);
      const int ex = wave_incl_scan(occ) - occ;
      compact_hash_runs<SRT, V>(t.keys, t.vals, TC, ex, c0, c1, ob, A.val, B.val, out.row, out.val);
    }
    wave_sync();
  }
}

// ---- block numeric: one item per workgroup
template <class SRT, typename V, int LOGT, int NT>
constexpr size_t num_block_lds() {
  return (size_t)((1 << LOGT) + NT) * (sizeof(typename SRT::Acc) + 4) + (size_t)NT * (20 + sizeof(V)) +
         (size_t)(NT / kWave + 1) * 8 + 64 * 4;
}

template <class SRT, typename V, int LOGT, int NT, bool UNIT>
__global__ void __launch_bounds__(NT) k_num_block(const int32_t* __restrict__ list, const int* __restrict__ count_dev,
                                                  int64_t count_host, const Unit* __restrict__ units, DevCsc<V> A,
                                                  DevCsc<V> B, const int2* __restrict__ span,
                                                  const int64_t* __restrict__ colptr, Split spl, NumOut<V> out) {
  using Acc = typename SRT::Acc;
  constexpr int T = 1 << LOGT;
  constexpr int TC = T + NT;      // tail = one slot per thread keeps chunks uniform
  extern __shared__ __attribute__((aligned(16))) char smem[];
  Acc* vals = (Acc*)smem;                        // TC
  int64_t* qb = (int64_t*)(vals + TC);           // NT   (Acc is 4 or 8 bytes and TC is even)
  int64_t* off = qb + NT;                        // NT
  int64_t* scr = off + NT;                       // NT/64 + 1
  int32_t* lens = (int32_t*)(scr + NT / kWave + 1); // NT
  V* bvs = (V*)(lens + NT);                      // NT
  int32_t* keys = (int32_t*)(bvs + NT);          // TC
  int* misc = keys + TC;                         // [1] overflow, [2] adderr, [8..] int scan
  Table<Acc> t{keys, vals, T, TC};
  const SegBuf<V> sb{qb, off, bvs, scr, lens};
  const int64_t count = count_dev ? (int64_t)*count_dev : count_host;
  for (int64_t i = blockIdx.x; i < count; i += gridDim.x) {
    const Work wk = get_work<UNIT>(list, i, units, span, colptr, spl.log);
    const int64_t spn = (int64_t)wk.hi - wk.lo + 1;
    const bool dense = spn <= T;
    const uint32_t mult = dense ? 0u : (uint32_t)(((uint64_t)T << 32) / (uint64_t)spn);
    for (int s = threadIdx.x; s < TC; s += NT) { keys[s] = dense ? 0 : kEmpty; vals[s] = SRT::identity(); }
    if (threadIdx.x == 0) { misc[1] = 0; misc[2] = 0; }
    __syncthreads();
    int ovf = 0, aerr = 0;
    for_each_multiply<NT, false, kUnroll, kGroupNum, V>(
        B.cp[wk.j], B.cp[wk.j + 1], sb,
        [&](int64_t b, int64_t& a0, int64_t& a1, V& bv) { num_seg<V, UNIT>(A, B, spl, spl.useg, wk, b, a0, a1, bv); },
        [&](int64_t q) { return NumItem<V>{A.ir[q], load_val(A.val, q)}; },
        [&](const NumItem<V>& it, V bv, int64_t q, int64_t b) {
          num_insert<SRT, V, UNIT>(t, dense, wk, mult, it, bv, q, b, ovf, aerr);
        });
    if (ovf) misc[1] = 1;
    if (aerr) misc[2] = 1;
    __syncthreads();
    const int64_t ob = wk.ob;
    if (misc[1]) {
      if (threadIdx.x == 0) out.ovf_list[atomicAdd(out.ovf_n, 1)] = list[i];
    } else if (dense) {
      constexpr int NWORD = T / 32;
      static_assert(NWORD <= NT, "dense bitmap words must not exceed the block");
      uint32_t wd = (threadIdx.x < NWORD) ? (uint32_t)keys[threadIdx.x] : 0u;
      int tot;
      int o = block_excl_scan<NT>(__popc(wd), misc + 8, &tot);
      while (wd) {
        const int bpos = __ffs(wd) - 1;
        wd &= wd - 1;
        const int rr = threadIdx.x * 32 + bpos;
        out.row[ob + o] = wk.lo + rr;
        out.val[ob + o] = SRT::out(vals[rr], A.val, B.val);
        ++o;
      }
    } else {
      // home counters in the (now idle) segment staging arrays: T/2 words <= 2*NT int64 slots
      static_assert((1 << LOGT) * 2 <= NT * 16, "home counters must fit the segment arrays");
      uint32_t* hc = (uint32_t*)qb;
      for (int w2 = threadIdx.x; w2 < T / 2; w2 += NT) hc[w2] = 0u;
      __syncthreads();
      compact_hash_homes<SRT, V, NT, TC / NT>(keys, vals, TC, T, wk.lo, mult, hc, misc + 8, ob, A.val, B.val,
                                              out.row, out.val);
    }
    if (threadIdx.x == 0 && misc[2]) atomicOr(out.adderr, 1);
    __syncthreads();
  }
}

// ---- heavy numeric: one workgroup per item = up to kItemUnits consecutive units of one heavy column.
// The item's unit descriptors are loaded once, and each unit's segments come from the precomputed
// table (k_unit_segs), fetched one chunk ahead so that the fetch overlaps the current expansion.
// Hash tables are sized per unit (power of two >= 2*cnt, >= NT) inside the T-slot allocation.
struct HeavyItem {
  int32_t h, u0, u1, pad;   // units [u0, u1) of heavy column h
};

template <class SRT, typename V, int LOGT, int NT>
constexpr size_t num_heavy_lds() {
  return num_block_lds<SRT, V, LOGT, NT>() + kItemUnits * (sizeof(Unit) + sizeof(UnitRows)) + (size_t)(1 << LOGT) * 2;
}

template <class SRT, typename V, int LOGT, int NT>
__global__ void __launch_bounds__(NT) k_num_heavy(const HeavyItem* __restrict__ items,
                                                  const unsigned long long* __restrict__ nitems,
                                                  const int32_t* __restrict__ hcols, const Unit* __restrict__ units,
                                                  int32_t nsub, DevCsc<V> A, DevCsc<V> B,
                                                  const int2* __restrict__ span, Split spl, NumOut<V> out,
                                                  unsigned long long* __restrict__ ticket) {
  using Acc = typename SRT::Acc;
  constexpr int T = 1 << LOGT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ unsigned long long s_claim;
  // vals and keys are adjacent: rank mode uses the pair as one region (values, then the bitmap)
  int64_t* qb = (int64_t*)smem;                  // NT
  int64_t* off = qb + NT;                        // NT
  int64_t* scr = off + NT;                       // NT/64 + 1
  V* bvs = (V*)(scr + NT / kWave + 1);           // NT
  int32_t* lens = (int32_t*)(bvs + NT);          // NT
  int* misc = lens + NT;                         // [1] overflow, [2] adderr, [8..] int scan (64 ints)
  Unit* s_units = (Unit*)(misc + 64);            // kItemUnits
  Acc* vals = (Acc*)(s_units + kItemUnits);      // T + NT
  int32_t* keys = (int32_t*)(vals + T + NT);     // T + NT
  uint32_t* hc = (uint32_t*)(keys + T + NT);     // T/2 packed home counters (compaction) / rank directory
  static_assert(sizeof(Unit) % 8 == 0 && sizeof(UnitRows) % 8 == 0 && (NT % 2) == 0,
                "LDS carve-up must keep 8-byte alignment");
  constexpr int64_t kRankBytes = (int64_t)(T + NT) * (int64_t)(sizeof(Acc) + 4);
  const SegBuf<V> sb{qb, off, bvs, scr, lens};
  STAMP_DECL
  STAMP(0);
  const int64_t nit = (int64_t)*nitems;   // persistent: items from the ticket (or b, b+G, ... when static)
  auto claim = [&](int64_t prev) -> int64_t {
    if (!CBG_HEAVY_DYNAMIC) return prev < 0 ? (int64_t)blockIdx.x : prev + gridDim.x;
    if (threadIdx.x == 0) s_claim = atomicAdd(ticket, 1ull);
    __syncthreads();
    const int64_t v = (int64_t)s_claim;
    __syncthreads();
    return v;
  };
  for (int64_t ii = claim(-1); ii < nit; ii = claim(ii)) {
  const HeavyItem item = items[ii];
  const int32_t j = hcols[item.h];
  const int2 sp = span[j];
  const int64_t bs = B.cp[j], nb = B.cp[j + 1] - bs;
  const int nu = item.u1 - item.u0;
  if ((int)threadIdx.x < nu) s_units[threadIdx.x] = units[(int64_t)item.h * nsub + item.u0 + threadIdx.x];
  __syncthreads();
  auto fetch = [&](int u, int64_t c, int64_t& a0, int64_t& a1, V& bv) {
    const int64_t i = c + threadIdx.x;
    a0 = a1 = 0;
    bv = V(0);
    if (u < nu && i < nb) {
      const UnitSeg g = spl.useg[s_units[u].segbase + i];
      a0 = g.a0;
      a1 = g.a1;
      bv = load_val(B.val, bs + i);
    }
  };
  int64_t pa0, pa1;
  V pbv;
  fetch(0, 0, pa0, pa1, pbv);
  STAMP(1);
  for (int u = 0; u < nu; ++u) {
    const Unit un = s_units[u];
    Work wk;
    wk.j = j;
    wk.s0 = un.s0;
    wk.s1 = un.s1;
    wk.lo = (int32_t)max((int64_t)sp.x, (int64_t)un.s0 << spl.log);
    wk.hi = (int32_t)min((int64_t)sp.y, ((int64_t)un.s1 << spl.log) - 1);
    wk.ob = un.outoff;
    wk.segbase = un.segbase;
    const int64_t spn = (int64_t)wk.hi - wk.lo + 1;
    const bool dense = spn <= T;
    int Te = NT;
    while (Te < T && Te < 2 * un.cnt) Te <<= 1;
    const int TC = Te + NT;
    const uint32_t mult = dense ? 0u : (uint32_t)(((uint64_t)Te << 32) / (uint64_t)spn);
    Table<Acc> t{keys, vals, Te, TC};
    // rank mode: presence bitmap of the unit's span (keys, <= T+NT words) + per-word rank directory
    // (16-bit, in hc: <= T words) give every output row its exact slot; no probing, no sort.
    // (values: cnt slots; bitmap: nw words right after them in the vals+keys region; directory: one
    // 16-bit prefix per word PAIR in hc, T entries -> spans up to 64*T rows)
    const int nw = (int)min<int64_t>((spn + 31) >> 5, 1 << 30);
    const int cpad = (un.cnt + 1) & ~1;
    const bool rank = CBG_RANK_MODE && !SRT::kAddIsError && !dense && un.cnt <= T &&
                      nw <= 2 * T && (int64_t)cpad * (int64_t)sizeof(Acc) + 4LL * nw <= kRankBytes;
    uint32_t* bm = (uint32_t*)(vals + cpad);
    if (dense) {
      for (int s = threadIdx.x; s < T / 32; s += NT) keys[s] = 0;
      for (int s = threadIdx.x; s < spn; s += NT) vals[s] = SRT::identity();
    } else if (rank) {
      for (int s = threadIdx.x; s < nw; s += NT) bm[s] = 0u;
      for (int s = threadIdx.x; s < un.cnt; s += NT) vals[s] = SRT::identity();
    } else {
      for (int s = threadIdx.x; s < TC; s += NT) { keys[s] = kEmpty; vals[s] = SRT::identity(); }
      for (int s = threadIdx.x; s < (Te >> 1); s += NT) hc[s] = 0u;
    }
    if (threadIdx.x == 0) { misc[1] = 0; misc[2] = 0; }
    __syncthreads();
    STAMP(2);
    STAMP_COUNT(10, 1);
    int ovf = 0, aerr = 0;
    uint16_t* pre = (uint16_t*)hc;
    auto mark = [&](int64_t F, int64_t c, int ns) {   // sweep 1: mark the rows (row ids only)
      expand_staged<NT, kUnrollHeavy, kGroupHeavy, V>(
          sb, threadIdx.x, F, bs + c, ns, [&](int64_t q) { return A.ir[q]; },
          [&](int32_t r, V, int64_t, int64_t) {
            if (r < wk.lo || r > wk.hi) return;
            const int o = r - wk.lo;
            atomicOr(&bm[o >> 5], 1u << (o & 31));
          });
    };
    auto accum = [&](int64_t F, int64_t c, int ns) {  // sweep 2: accumulate at the exact slots
      expand_staged<NT, kUnrollHeavy, kGroupHeavy, V>(
          sb, threadIdx.x, F, bs + c, ns, [&](int64_t q) { return NumItem<V>{A.ir[q], load_val(A.val, q)}; },
          [&](const NumItem<V>& it, V bv2, int64_t q, int64_t b) {
            if (it.r < wk.lo || it.r > wk.hi) return;
            const int o = it.r - wk.lo, w = o >> 5;
            const int slot = (int)pre[w >> 1] + ((w & 1) ? __popc(bm[w - 1]) : 0) +
                             __popc(bm[w] & ((1u << (o & 31)) - 1u));
            SRT::acc(&vals[slot], SRT::mul(it.a, bv2, q, b));
          });
    };
    // rank directory: exclusive popcount prefix per word pair (contiguous even word ranges per
    // thread); false if the bitmap disagrees with the symbolic count (cannot happen: it is exact)
    auto directory = [&]() -> bool {
      const int WPT = (((nw + NT - 1) / NT) + 1) & ~1;
      const int w0 = min(nw, (int)threadIdx.x * WPT), w1 = min(nw, w0 + WPT);
      int local = 0;
      for (int w = w0; w < w1; ++w) local += __popc(bm[w]);
      int tot;
      int run = block_excl_scan<NT>(local, misc + 8, &tot);
      for (int w = w0; w < w1; ++w) {
        if (!(w & 1)) pre[w >> 1] = (uint16_t)run;
        run += __popc(bm[w]);
      }
      __syncthreads();
      return tot == un.cnt;
    };
    // a multi-chunk rank unit streams its segments twice (mark pass, then accumulate pass); a
    // single-chunk one stages them once and runs both sweeps on the staged chunk
    const bool multi = rank && nb > NT;
    for (int pass = 0; pass < (multi ? 2 : 1); ++pass) {
      for (int64_t c = 0; c < nb; c += NT) {
        const int64_t a0 = pa0, a1 = pa1;
        const V bv = pbv;
        if (c + NT < nb) fetch(u, c + NT, pa0, pa1, pbv);
        else if (multi && pass == 0) fetch(u, 0, pa0, pa1, pbv);
        else fetch(u + 1, 0, pa0, pa1, pbv);
        const int64_t F = stage_segments<NT, false, kGroupHeavy, V>(sb, a0, a1, bv);
        const int ns = (int)min<int64_t>(NT, nb - c);
        STAMP(3);
        STAMP_COUNT(11, 1);
        STAMP_COUNT(12, F);
        if (!rank) {
          expand_staged<NT, kUnrollHeavy, kGroupHeavy, V>(
              sb, threadIdx.x, F, bs + c, ns, [&](int64_t q) { return NumItem<V>{A.ir[q], load_val(A.val, q)}; },
              [&](const NumItem<V>& it, V bv2, int64_t q, int64_t b) {
                num_insert<SRT, V, true>(t, dense, wk, mult, it, bv2, q, b, ovf, aerr);
              });
        } else if (!multi && F <= (int64_t)NT * kUnrollHeavy * CBG_RANK_REGS) {
          const bool ok = expand_staged_twice<NT, kUnrollHeavy, kGroupHeavy, CBG_RANK_REGS, V>(
              sb, threadIdx.x, F, bs + c, ns, [&](int64_t q) { return A.ir[q]; },
              [&](int64_t q) { return load_val(A.val, q); },
              [&](int32_t r) {
                if (r < wk.lo || r > wk.hi) return;
                const int o = r - wk.lo;
                atomicOr(&bm[o >> 5], 1u << (o & 31));
              },
              [&]() {
                __syncthreads();
                STAMP(24);
                const bool d = directory();
                STAMP(25);
                return d;
              },
              [&](int32_t r, V a, V bv2, int64_t q, int64_t b) {
                if (r < wk.lo || r > wk.hi) return;
                const int o = r - wk.lo, w = o >> 5;
                const int slot = (int)pre[w >> 1] + ((w & 1) ? __popc(bm[w - 1]) : 0) +
                                 __popc(bm[w] & ((1u << (o & 31)) - 1u));
                SRT::acc(&vals[slot], SRT::mul(a, bv2, q, b));
              });
          if (!ok) ovf = 1;
        } else if (!multi) {
          mark(F, c, ns);
          __syncthreads();
          if (directory()) accum(F, c, ns);
          else ovf = 1;
        } else if (pass == 0) {
          mark(F, c, ns);
        } else {
          accum(F, c, ns);
        }
        __syncthreads();
        STAMP(4);
      }
      if (multi && pass == 0 && !directory()) {
        ovf = 1;
        fetch(u + 1, 0, pa0, pa1, pbv);   // the prefetched chunk was this unit's: take the next unit's
        break;
      }
    }
    if (ovf) misc[1] = 1;
    if (aerr) misc[2] = 1;
    __syncthreads();
    STAMP(6);
    const int64_t ob = wk.ob;
    if (misc[1]) {
      if (threadIdx.x == 0) out.ovf_list[atomicAdd(out.ovf_n, 1)] = (int32_t)((int64_t)item.h * nsub + item.u0 + u);
    } else if (dense) {
      constexpr int NWORD = T / 32;
      static_assert(NWORD <= NT, "dense bitmap words must not exceed the block");
      uint32_t wd = (threadIdx.x < NWORD) ? (uint32_t)keys[threadIdx.x] : 0u;
      int tot;
      int o = block_excl_scan<NT>(__popc(wd), misc + 8, &tot);
      while (wd) {
        const int bpos = __ffs(wd) - 1;
        wd &= wd - 1;
        const int rr = threadIdx.x * 32 + bpos;
        out.row[ob + o] = wk.lo + rr;
        out.val[ob + o] = SRT::out(vals[rr], A.val, B.val);
        ++o;
      }
    } else if (rank) {
      // rows: word w's set bits go to pre[w].. in bit order (interleaved words: neighbouring lanes
      // write neighbouring positions); values: the slot array is already in row order
      const uint16_t* pre = (const uint16_t*)hc;
      for (int w = threadIdx.x; w < nw; w += NT) {
        uint32_t wd = bm[w];
        int o = (int)pre[w >> 1] + ((w & 1) ? __popc(bm[w - 1]) : 0);
        while (wd) {
          const int bpos = __ffs(wd) - 1;
          wd &= wd - 1;
          out.row[ob + o] = wk.lo + w * 32 + bpos;
          ++o;
        }
      }
      for (int i = threadIdx.x; i < un.cnt; i += NT) out.val[ob + i] = SRT::out(vals[i], A.val, B.val);
    } else {
      STAMP(7);
      compact_hash_homes<SRT, V, NT, T / NT + 1>(keys, vals, TC, Te, wk.lo, mult, hc, misc + 8, ob,
                                                A.val, B.val, out.row, out.val);
      STAMP(8);
      STAMP_COUNT(13, 1);
    }
    if (threadIdx.x == 0 && misc[2]) atomicOr(out.adderr, 1);
    __syncthreads();
    STAMP(5);
  }
  }
}

// ---- heavy numeric with the rows known (symbolic row handoff).  A persistent kernel: workgroup b
// takes the rows-known units b, b+G, b+2G, ... of one flat list (KnownUnit, built by
// k_heavy_items_split), keeping the next unit's header and sorted rows in flight while it sweeps the
// current one.  Per unit:
//   a. its sorted output rows (symbolic scratch pieces, prefetched into registers) go to C.row; for every 64-row pair holding rows the pair's first row clears the two
//      bitmap words and records its rank (pre[pair]); the value slots are cleared;
//   b. every row sets its bit -- words of empty pairs are never read, so nothing span-sized is cleared
//      or scanned;
//   c. ONE sweep over the multiplies: gather (row, value), slot = pre[pair] + popcount of the pair word
//      below the row, SR::acc at that slot (exact: every gathered row of the unit's range is an output
//      row);
//   d. the values, already in row order, are written out.
// rows per thread of k_num_heavy_known (a multi-subwindow unit has at most kUnitCap outputs)
template <int NT>
constexpr int known_rpt() { return (int)((kUnitCap + NT - 1) / NT); }

template <class SRT, int LOGT, int NT>
__device__ __forceinline__ bool heavy_unit_known(const Unit& un, int2 usp, const UnitRows& ur) {
  using Acc = typename SRT::Acc;
  constexpr int T = 1 << LOGT;
  constexpr int64_t kRankBytes = (int64_t)(T + NT) * (int64_t)(sizeof(Acc) + 4);
  const int64_t spn = (int64_t)usp.y - usp.x + 1;
  const int64_t nw = (spn + 31) >> 5;
  const int64_t cpad = (un.cnt + 1) & ~1;
  // nw <= 2T also bounds the span to 64T = 2^19 rows
  return !SRT::kAddIsError && CBG_RANK_MODE && ur.np >= 1 && ur.np <= 3 && spn > T && un.cnt <= T &&
         un.cnt <= known_rpt<NT>() * NT && nw <= 2 * (int64_t)T &&
         cpad * (int64_t)sizeof(Acc) + 4 * (nw + 1) <= kRankBytes;
}

// everything k_num_heavy_known needs about one unit, in one 72-byte record
struct KnownUnit {
  int64_t outoff;       // first output in C
  int64_t segbase;      // the unit's (unit, B nonzero) segments in Split::useg
  int64_t bs;           // B.cp[j]
  int64_t roff[3];      // row pieces in the symbolic row scratch (Split::hrows)
  int32_t o1, o2;       // ranks where pieces 1 and 2 start (o1 = o2 = cnt: one piece)
  int32_t cnt, nb;      // outputs; B nonzeros of the column
  int32_t lo, hi;       // the unit's row range [lo, hi]
};
static_assert(sizeof(KnownUnit) == 72, "KnownUnit is 18 words");
constexpr int kKnownWords = (int)(sizeof(KnownUnit) / 4);

__device__ __forceinline__ int64_t known_row_src(const KnownUnit& H, int i) {
  return i < H.o1 ? H.roff[0] + i : i < H.o2 ? H.roff[1] + (i - H.o1) : H.roff[2] + (i - H.o2);
}

// The rows-known kernel takes its units from a device ticket (CBG_HEAVY_DYNAMIC), claiming unit k+3 at the top of unit k
// and publishing it at the end, so the atomic's round trip is never waited on.  The claim goes through an address the
// compiler cannot prove uniform: the atomic optimizer's wave-aggregated form needs the old value at once (an s_waitcnt at
// the top of every unit; s20 heavy 31.1 -> 31.0 ms, profiles/r05g_variants_s20.txt).  C is written with nontemporal
// stores, streamed past the L2 that serves A's gathers (s20 heavy 31.1 -> 30.4 ms, same file).  Measured and removed in
// round 6 (git history): claiming two ahead, paired 16-byte value stores (no change either way).
static_assert(CBG_HEAVY_DYNAMIC, "k_num_heavy_known claims its units from the device ticket");
// k_num_heavy_known: groups of CBG_GROUP_KNOWN entries, CBG_UNROLL_KNOWN groups in flight per lane
// (s20 f64: G=2/U=4 32.4 ms, G=4/U=2 34.5, G=1/U=8 38.1, G=8/U=1 41.4; G=4/U=3 spills)
#ifndef CBG_UNROLL_KNOWN
#define CBG_UNROLL_KNOWN 4
#endif
#ifndef CBG_GROUP_KNOWN
#define CBG_GROUP_KNOWN 2
#endif

// A's (row, value) pairs interleaved for the heavy gathers: one 16-byte (8-byte for 4-byte values) load per
// multiply instead of a row load and a value load
template <typename V> struct alignas(sizeof(V) == 8 ? 16 : 8) RowVal {
  int32_t r;
  int32_t pad_[sizeof(V) == 8 ? 1 : 0];
  V v;
};
template <typename V>
__global__ void k_pack_rowval(int64_t nnz, const int32_t* __restrict__ ir, const V* __restrict__ val,
                              RowVal<V>* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nnz; i += (int64_t)gridDim.x * blockDim.x) {
    RowVal<V> e;
    e.r = ir[i];
    e.v = val[i];
    out[i] = e;
  }
}

template <class SRT, typename V, int LOGT, int NT, bool AV, bool AOS = false>
__global__ void __launch_bounds__(NT) k_num_heavy_known(const KnownUnit* __restrict__ ku,
                                                        const unsigned long long* __restrict__ nku, DevCsc<V> A,
                                                        DevCsc<V> B, Split spl, NumOut<V> out,
                                                        unsigned long long* __restrict__ ticket,
                                                        const RowVal<V>* __restrict__ arv = nullptr) {
  using Acc = typename SRT::Acc;
  constexpr int T = 1 << LOGT;
  constexpr int RPT = known_rpt<NT>();   // rows per thread (cnt <= RPT*NT)
  constexpr int NW = NT / kWave;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int64_t* qb = (int64_t*)smem;                  // NT
  int64_t* off = qb + NT;                        // NT
  int64_t* scr = off + NT;                       // NT/64 + 1
  V* bvs = (V*)(scr + NT / kWave + 1);           // NT
  int32_t* lens = (int32_t*)(bvs + NT);          // NT
  KnownUnit* hdr = (KnownUnit*)(lens + NT);      // 2: this unit's and the next unit's header (ring)
  int32_t* bnd = (int32_t*)(hdr + 2);            // NW*RPT (+1 pad): the last row of every wave, per q
  Acc* vals = (Acc*)(bnd + ((NW * RPT + 1) & ~1)); // (T + NT) * (sizeof(Acc) + 4) bytes: values, then the bitmap
  uint16_t* pre = (uint16_t*)((char*)vals + (size_t)(T + NT) * (sizeof(Acc) + 4));   // T entries
  static_assert((NT % 2) == 0, "LDS carve-up must keep 8-byte alignment");
  const SegBuf<V> sb{qb, off, bvs, scr, lens};
  const int tid = threadIdx.x;
  const int64_t n = (int64_t)*nku;
  // units k (current), k1 (next: header and rows in flight), k2 (claimed one unit earlier, header loaded during unit
  // k); unit k3 is claimed at the top of unit k and its number published at the end of it
  __shared__ unsigned long long s_claim;
  if (tid == 0) s_claim = atomicAdd(ticket, 3ull);
  __syncthreads();
  int64_t k = (int64_t)s_claim, k1 = k + 1, k2 = k + 2;
  if (k >= n) return;   // uniform
  STAMP_DECL
  STAMP(0);
  const uint32_t* kw = (const uint32_t*)ku;
  uint32_t* hw = (uint32_t*)hdr;
  if (tid < kKnownWords) {
    hw[tid] = kw[k * kKnownWords + tid];
    if (k1 < n) hw[kKnownWords + tid] = kw[k1 * kKnownWords + tid];
  }
  __syncthreads();
  int32_t rr[RPT];
  // rows i = tid + q*NT (coalesced; clamped loads): the loads stay in flight during the current unit's sweep
  auto load_rows = [&](const KnownUnit& H) {
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      const int i = tid + q * NT;
      rr[q] = spl.hrows[known_row_src(H, i < H.cnt ? i : 0)];
    }
  };
  // every wave's last row per q, for the pair-boundary test of the next wave's first lane
  const int lane = lane_id(), wv = tid / kWave;
  auto put_bnd = [&]() {
    if (lane == kWave - 1) {
#pragma unroll
      for (int q = 0; q < RPT; ++q) bnd[wv * RPT + q] = rr[q];
    }
  };
  auto fetch = [&](const KnownUnit& H, int64_t c, int64_t& a0, int64_t& a1, V& bv) {
    const int64_t i = c + tid;
    a0 = a1 = 0;
    bv = V(0);
    if (i < H.nb) {
      const UnitSeg g = spl.useg[H.segbase + i];
      a0 = g.a0;
      a1 = g.a1;
      bv = load_val(B.val, H.bs + i);
    }
  };
  int64_t pa0, pa1;
  V pbv;
  {
    const KnownUnit H0 = hdr[0];
    load_rows(H0);
    fetch(H0, 0, pa0, pa1, pbv);
    put_bnd();
    __syncthreads();
  }
  for (int slot = 0; k < n; slot ^= 1) {
    STAMP(1);
    const KnownUnit H = hdr[slot];
    const bool has1 = k1 < n;
    unsigned long long k3 = 0;
    // through an address the compiler cannot prove uniform: the atomic optimizer's wave-aggregated form needs the old
    // value right away (an s_waitcnt on the atomic at the top of every unit); this plain form waits only where k3 is
    // used, at the end of the unit
    if (tid == 0) {
      int32_t z;
      asm volatile("v_mov_b32 %0, 0" : "=v"(z));
      k3 = atomicAdd(ticket + z, 1ull);
    }
    const int32_t lo = __builtin_amdgcn_readfirstlane(H.lo), hi = __builtin_amdgcn_readfirstlane(H.hi);
    const int32_t cnt = __builtin_amdgcn_readfirstlane(H.cnt);
    const int cpad = (cnt + 1) & ~1;
    uint32_t* bm = (uint32_t*)(vals + cpad);
    // a. value slots cleared; rows -> C.row; the first row of each pair clears the pair, records its rank
    for (int i = tid; i < cnt; i += NT) vals[i] = SRT::identity();
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      const int i = tid + q * NT;
      const int32_t r = rr[q];
      const int32_t up = __shfl_up(r, 1, kWave);   // row i-1 within the wave
      if (i < cnt) {
        __builtin_nontemporal_store(r, &out.row[H.outoff + i]);
        const int pr = (r - lo) >> 6;
        const int32_t p = lane ? up : (wv ? bnd[(wv - 1) * RPT + q] : (q ? bnd[(NW - 1) * RPT + q - 1] : r));
        if (i == 0 || ((p - lo) >> 6) != pr) {
          bm[2 * pr] = 0u;
          bm[2 * pr + 1] = 0u;
          pre[pr] = (uint16_t)i;
        }
      }
    }
    STAMP(6);
    __syncthreads();
    STAMP(7);
    const bool has2 = k2 < n;
    uint32_t nh = 0;   // header of unit k2, written to this unit's ring slot at the end
    if (tid < kKnownWords && has2) nh = kw[k2 * kKnownWords + tid];
    // b. bits
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      const int i = tid + q * NT;
      if (i < cnt) {
        const int o = rr[q] - lo;
        atomicOr(&bm[o >> 5], 1u << (o & 31));
      }
    }
    STAMP(8);
    if (has1) load_rows(hdr[slot ^ 1]);   // next unit's rows: in flight during the sweep
    STAMP(9);
    __syncthreads();
    STAMP(2);
    // c. one sweep over the unit's multiplies
    const uint64_t* bm2 = (const uint64_t*)bm;
    for (int64_t c = 0; c < H.nb; c += NT) {
      const int64_t a0 = pa0, a1 = pa1;
      const V bv = pbv;
      if (c + NT < H.nb) fetch(H, c + NT, pa0, pa1, pbv);
      else if (has1) fetch(hdr[slot ^ 1], 0, pa0, pa1, pbv);
      const int64_t F = stage_segments<NT, false, CBG_GROUP_KNOWN, V>(sb, a0, a1, bv);
      STAMP(3);
      auto ld_one = [&](int64_t q) {   // AV: no pointer test per load; AOS: one load for the row and the value
            if constexpr (AOS && sizeof(V) == 8) {   // one dwordx4: (row, pad, value)
              typedef int v4i __attribute__((ext_vector_type(4)));
              const v4i w = *(const v4i*)(arv + q);
              const long long b = ((long long)(unsigned)w.w << 32) | (unsigned)w.z;
              V v;
              __builtin_memcpy(&v, &b, 8);
              return NumItem<V>{w.x, v};
            } else if constexpr (AOS) {              // one dwordx2: (row, value)
              typedef int v2i __attribute__((ext_vector_type(2)));
              const v2i w = *(const v2i*)(arv + q);
              const int wy = w.y;
              V v;
              __builtin_memcpy(&v, &wy, sizeof(V) < 4 ? sizeof(V) : 4);
              return NumItem<V>{w.x, v};
            } else {
              return NumItem<V>{A.ir[q], AV ? A.val[q] : V(1)};
            }
          };
      auto slotf = [&](const NumItem<V>& it) -> int {
            const uint32_t o = (uint32_t)(it.r - lo);
            const bool ok = o <= (uint32_t)(hi - lo);
            const uint32_t oc = ok ? o : 0u;
            const int sl = (int)pre[oc >> 6] + __popcll(bm2[oc >> 6] & ((1ull << (oc & 63)) - 1ull));
            return ok ? sl : -1;
          };
      auto accf = [&](int sl, const NumItem<V>& it, V bv2, int64_t q, int64_t b) {
            SRT::acc(&vals[sl], SRT::mul(it.a, bv2, q, b));
          };
      const NumLd2<V, AV> ld2{A.ir, A.val, A.nnz};
      if constexpr (!AOS && CBG_NUM_VEC2 && CBG_GROUP_KNOWN == 2) {
        if (A.nnz >= 2)   // uniform
          expand_staged_slots<NT, CBG_UNROLL_KNOWN, CBG_GROUP_KNOWN, V>(sb, tid, F, H.bs + c,
                                                                      (int)min<int64_t>(NT, H.nb - c), ld2, slotf, accf);
        else
          expand_staged_slots<NT, CBG_UNROLL_KNOWN, CBG_GROUP_KNOWN, V>(sb, tid, F, H.bs + c,
                                                                      (int)min<int64_t>(NT, H.nb - c), ld_one, slotf, accf);
      } else {
        expand_staged_slots<NT, CBG_UNROLL_KNOWN, CBG_GROUP_KNOWN, V>(sb, tid, F, H.bs + c,
                                                                    (int)min<int64_t>(NT, H.nb - c), ld_one, slotf, accf);
      }
      __syncthreads();
      STAMP(4);
    }
    // d. values out, row order
    for (int i = tid; i < cnt; i += NT) __builtin_nontemporal_store(SRT::out(vals[i], A.val, B.val), &out.val[H.outoff + i]);
    STAMP(10);
    if (tid < kKnownWords && has2) hw[slot * kKnownWords + tid] = nh;
    if (has1) put_bnd();
    if (tid == 0) s_claim = k3;
    __syncthreads();
    STAMP(5);
    k = k1;
    k1 = k2;
    k2 = (int64_t)s_claim;   // k3: published before the barrier above; rewritten only after the next one
  }
}

template <class SRT, typename V, int LOGT, int NT>
constexpr size_t num_heavy_known_lds() {
  return (size_t)NT * (8 + 8 + sizeof(V) + 4) + (size_t)(NT / kWave + 1) * 8 + 2 * sizeof(KnownUnit) +
         (size_t)(((NT / kWave) * known_rpt<NT>() + 1) & ~1) * 4 +
         (size_t)((1 << LOGT) + NT) * (sizeof(typename SRT::Acc) + 4) + (size_t)(1 << LOGT) * 2;
}

// Every heavy column's units -> the rows-known list (one KnownUnit per eligible unit, for
// k_num_heavy_known) and items for k_num_heavy (runs of consecutive other units, <= kItemUnits per
// item); list lengths -> counts[0], counts[1].  Runs after k_unit_segs (segbase).
template <class SRT, int LOGT, int NT>
__global__ void k_heavy_items_split(int H, const int32_t* __restrict__ cols, const int32_t* __restrict__ nunits,
                                    const Unit* __restrict__ units, int32_t nsub, int32_t log,
                                    const int32_t* __restrict__ sub, const int2* __restrict__ uspan,
                                    const UnitRows* __restrict__ urows, const int64_t* __restrict__ Bcp,
                                    KnownUnit* __restrict__ known, HeavyItem* __restrict__ oitems,
                                    unsigned long long* __restrict__ counts) {
  const int h = blockIdx.x * blockDim.x + threadIdx.x;
  const int nu = h < H ? nunits[h] : 0;
  auto is_known = [&](int u) {
    const int64_t slot = (int64_t)h * nsub + u;
    return urows != nullptr && heavy_unit_known<SRT, LOGT, NT>(units[slot], uspan[slot], urows[slot]);
  };
  int nk = 0, no = 0;
  for (int u = 0, run = 0; u < nu; ++u) {
    if (is_known(u)) { ++nk; run = 0; }
    else { if (run == 0) ++no; if (++run == kItemUnits) run = 0; }
  }
  // one atomic per wave and list (a single counter hit by every column serialises at the L2)
  const int ik = wave_incl_scan(nk), io = wave_incl_scan(no);
  unsigned long long bk = 0, bo = 0;
  if (lane_id() == kWave - 1) {
    bk = ik ? atomicAdd(&counts[0], (unsigned long long)ik) : 0;
    bo = io ? atomicAdd(&counts[1], (unsigned long long)io) : 0;
  }
  bk = __shfl(bk, kWave - 1, kWave) + (ik - nk);
  bo = __shfl(bo, kWave - 1, kWave) + (io - no);
  if (nu == 0) return;
  const int32_t j = cols[h];
  const int64_t bs = Bcp[j];
  const int32_t nb = (int32_t)(Bcp[j + 1] - bs);
  int u0 = -1;
  for (int u = 0; u < nu; ++u) {
    if (is_known(u)) {
      if (u0 >= 0) { oitems[bo++] = HeavyItem{h, u0, u, 0}; u0 = -1; }
      const int64_t slot = (int64_t)h * nsub + u;
      const Unit un = units[slot];
      const UnitRows ur = urows[slot];
      const int2 sp = uspan[slot];
      KnownUnit K;
      K.outoff = un.outoff;
      K.segbase = un.segbase;
      K.bs = bs;
      K.roff[0] = ur.off[0];
      K.roff[1] = ur.np > 1 ? ur.off[1] : 0;
      K.roff[2] = ur.np > 2 ? ur.off[2] : 0;
      K.o1 = ur.np > 1 ? ur.n[0] : un.cnt;
      K.o2 = ur.np > 2 ? ur.n[0] + ur.n[1] : un.cnt;
      K.cnt = un.cnt;
      K.nb = nb;
      K.lo = sp.x;
      K.hi = sp.y;
      known[bk++] = K;
    } else {
      if (u0 < 0) u0 = u;
      if (u + 1 - u0 == kItemUnits) { oitems[bo++] = HeavyItem{h, u0, u + 1, 0}; u0 = -1; }
    }
  }
  if (u0 >= 0) oitems[bo++] = HeavyItem{h, u0, nu, 0};
}

// Rows-known units in first-subwindow order (CBG_KNOWN_SORT): the persistent kernel takes its units in list order, so
// the units in flight together then cover one row range of many columns and gather only that range of the A columns
// they share, instead of every range of a few columns.  Counting sort over the subwindow buckets in chunks of 256
// units: a chunk's bucket counts in LDS, one global atomic per (chunk, bucket) -- not one per unit on a few hundred
// counters, which serialised at the L2 (round 4: 2.5 ms) -- and the units' ranks inside their chunk from LDS atomics.
constexpr int kSortChunk = 256;
template <bool SCATTER>
__global__ void __launch_bounds__(kSortChunk) k_known_bucket(const KnownUnit* __restrict__ in,
                                                             const unsigned long long* __restrict__ nknown, int32_t log,
                                                             int32_t nb, unsigned long long* __restrict__ bcnt,
                                                             const unsigned long long* __restrict__ bbase,
                                                             unsigned long long* __restrict__ bcur,
                                                             KnownUnit* __restrict__ out) {
  __shared__ int lh[kMaxSub];
  __shared__ unsigned long long lb[kMaxSub];
  const int64_t n = (int64_t)*nknown;
  for (int64_t c0 = (int64_t)blockIdx.x * kSortChunk; c0 < n; c0 += (int64_t)gridDim.x * kSortChunk) {
    for (int b = threadIdx.x; b < nb; b += kSortChunk) lh[b] = 0;
    __syncthreads();
    const int64_t i = c0 + threadIdx.x;
    int bk = -1, r = 0;
    if (i < n) {
      bk = min(nb - 1, max(0, in[i].lo >> log));
      r = atomicAdd(&lh[bk], 1);
    }
    __syncthreads();
    for (int b = threadIdx.x; b < nb; b += kSortChunk) {
      const int c = lh[b];
      if (c) {
        if (SCATTER) lb[b] = bbase[b] + atomicAdd(&bcur[b], (unsigned long long)c);
        else atomicAdd(&bcnt[b], (unsigned long long)c);
      }
    }
    if (SCATTER) {
      __syncthreads();
      if (i < n) out[lb[bk] + r] = in[i];
    }
    __syncthreads();
  }
}

// exclusive scan of the nb (<= kMaxSub) bucket counts, one workgroup
__global__ void __launch_bounds__(1024) k_known_bucket_base(int32_t nb, const unsigned long long* __restrict__ bcnt,
                                                            unsigned long long* __restrict__ bbase) {
  __shared__ int64_t scr[1024 / kWave + 1];
  constexpr int PER = (kMaxSub + 1023) / 1024;
  int64_t v[PER], t = 0;
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    const int b = threadIdx.x * PER + e;
    v[e] = b < nb ? (int64_t)bcnt[b] : 0;
    t += v[e];
  }
  int64_t tot;
  int64_t ex = block_excl_scan64<1024>(t, scr, &tot);
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    const int b = threadIdx.x * PER + e;
    if (b < nb) bbase[b] = (unsigned long long)ex;
    ex += v[e];
  }
}

// items of every heavy column: ceil(nunits / kItemUnits) consecutive unit groups
__global__ void k_heavy_items(int H, const int32_t* __restrict__ nunits, const int64_t* __restrict__ itemoff,
                              HeavyItem* __restrict__ items) {
  const int h = blockIdx.x * blockDim.x + threadIdx.x;
  if (h >= H) return;
  const int nu = nunits[h];
  int64_t o = itemoff[h];
  for (int u = 0; u < nu; u += kItemUnits) items[o++] = HeavyItem{h, u, min(nu, u + kItemUnits), 0};
}

// ============================================================================ 7. windowed sweep
// One workgroup per column, sweeping row windows [r0, r0+W) over the column's span.  Every B nonzero
// b owns a cursor into A(:,k) (cur[b], absolute index) and caches the row at the cursor (nxt[b]); a
// window only touches segments whose cached row is inside it.
//   MODE 0 = symbolic for spans wider than one 2^20-row bitmap: counts, and (the column is heavy)
//            nnz per subwindow;
//   MODE 1 = numeric fallback for whole columns whose order-preserving hash overflowed: dense value
//            window of 8192 rows + presence bitmap, compaction in row order.
constexpr int kWinRows = 8192;         // numeric dense window (64 KB of f64 values)
constexpr int kSymWinRows = 1 << 20;   // symbolic bitmap window (128 KB)

template <int MODE, class SRT, typename V, int NT, int W>
constexpr size_t window_lds() {
  return (MODE == 1 ? (size_t)W * sizeof(typename SRT::Acc) : 0) + (size_t)(W / 32) * 4 + (size_t)NT * 4 +
         (MODE == 0 ? (size_t)(W / kWinRows + 2) * 4 : 0) + 64 * 4;
}

template <int MODE, class SRT, typename V, int NT, int W>
__global__ void __launch_bounds__(NT) k_window(const int32_t* __restrict__ list, const int* __restrict__ count_dev,
                                               int64_t count_host, DevCsc<V> A, DevCsc<V> B,
                                               const int2* __restrict__ span, const int64_t* __restrict__ colptr,
                                               int64_t* __restrict__ cur, int32_t* __restrict__ nxt,
                                               int64_t* __restrict__ nnz, HeavyOut ho, NumOut<V> out) {
  using Acc = typename SRT::Acc;
  constexpr int NWORD = W / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  Acc* vals = (Acc*)smem;                                    // W (MODE 1) or 0
  uint32_t* bits = (uint32_t*)(vals + (MODE == 1 ? W : 0));  // NWORD
  int32_t* lq = (int32_t*)(bits + NWORD);                    // NT (queue of long segments)
  int32_t* scnt = lq + NT;                                   // MODE 0: subwindow counters
  int* misc = scnt + (MODE == 0 ? (W / kWinRows + 2) : 0);   // [0] lq n, [1] count, [2] adderr, [3] h, [8..] scan
  const int64_t count = count_dev ? (int64_t)*count_dev : count_host;
  for (int64_t i = blockIdx.x; i < count; i += gridDim.x) {
    const int32_t j = list[i];
    const int2 sp = span[j];
    const int64_t bs = B.cp[j], be = B.cp[j + 1];
    for (int64_t b = bs + threadIdx.x; b < be; b += NT) {
      const int32_t k = B.ir[b];
      const int64_t a0 = A.cp[k], a1 = A.cp[k + 1];
      cur[b] = a0;
      nxt[b] = a0 < a1 ? A.ir[a0] : INT32_MAX;
    }
    if (threadIdx.x == 0) {
      misc[2] = 0;
      if (MODE == 0) {
        const int h = atomicAdd(ho.n, 1);
        misc[3] = h;
        ho.cols[h] = j;
      }
    }
    __syncthreads();
    int64_t outpos = (MODE == 1) ? colptr[j] : 0;
    int64_t total = 0;
    int aerr = 0;
    // MODE 0 windows start on a subwindow boundary (W is a multiple of SUBW), so no subwindow's
    // count straddles two windows; MODE 1 windows only need 32-row alignment for the bitmap.
    const int32_t start = (MODE == 0) ? ((sp.x >> ho.log) << ho.log) : (sp.x & ~31);
    for (int64_t r0 = start; r0 <= sp.y; r0 += W) {
      const int32_t r1 = (int32_t)min<int64_t>(r0 + W, (int64_t)sp.y + 1);
      for (int s = threadIdx.x; s < NWORD; s += NT) bits[s] = 0u;
      if constexpr (MODE == 1)
        for (int s = threadIdx.x; s < W; s += NT) vals[s] = SRT::identity();
      __syncthreads();
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
              const int fl = __ffsll((long long)~m) - 1;
              rn = __shfl(r, fl, kWave);
              break;
            }
          }
          if (lane_id() == 0) { cur[sb] = sq; nxt[sb] = rn; }
        }
        __syncthreads();
      }
      int tot;
      if constexpr (MODE == 0) {
        // count + nnz per subwindow (windows start 32-aligned, so a word never straddles one)
        const int32_t sf = (int32_t)(r0 >> ho.log);
        const int nsw = (int)(((int64_t)r1 - 1) >> ho.log) - sf + 1;
        for (int s = threadIdx.x; s < nsw; s += NT) scnt[s] = 0;
        if (threadIdx.x == 0) misc[1] = 0;
        __syncthreads();
        int wcnt = 0;
        for (int s = threadIdx.x; s < NWORD; s += NT) {
          const int pc = __popc(bits[s]);
          if (pc) {
            wcnt += pc;
            atomicAdd(&scnt[((r0 + 32 * s) >> ho.log) - sf], pc);
          }
        }
        int64_t ws = wave_sum64(wcnt);
        if (lane_id() == 0 && ws) atomicAdd(&misc[1], (int)ws);
        __syncthreads();
        total += misc[1];
        int32_t* dst = ho.sub + (int64_t)misc[3] * ho.nsub;
        const int32_t slast = sp.y >> ho.log;
        for (int s = threadIdx.x; s < nsw; s += NT)
          if (sf + s <= slast) dst[sf + s] = scnt[s];
        __syncthreads();
      } else {
        constexpr int PW = NWORD / NT;
        static_assert(NWORD % NT == 0, "window words must split evenly");
        int c = 0;
        for (int s = 0; s < PW; ++s) c += __popc(bits[threadIdx.x * PW + s]);
        int o = block_excl_scan<NT>(c, misc + 8, &tot);
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
