// mcl.hip -- HipMCL column prune / select / recover and column split/concatenate on MI355X.
//
// Reference (include/CombBLAS): MCLPruneRecoverySelect ParFriends.h:185-353, Kselect1
// SpParMat.cpp:1413-1700 (k-th largest of a column; fewer than k entries -> the column minimum;
// empty -> numeric_limits<V>::min()), PruneColumn SpParMat.cpp:2567-2720 (drops v < threshold),
// Prune(bind2nd(less_equal, thr)) for the column statistics (drops v <= thr), ColSplit
// SpDCCols.cpp:927-1086 and ColConcatenate SpDCCols.cpp:1087-1185 (MemEfficientSpGEMM phases,
// ParFriends.h:449-730).
//
// Per output column j with values v (one column of the local matrix, all of its rows present):
//   nU = |v|, P = {v > thr}, nP = |P|, sP = sum(P)
//   recover : nP < R && nU > nP && sP < pct                    -> th = kth(v, R)
//   select  : !recover && S > 0 && nP > S                       -> th = kth(v, S); then if R > 0:
//             n1 = |{v >= th}|, s1 = sum{v >= th}; n1 < R && s1 < pct -> th = kth(v, R)
//   else    : th = thr
//   keep v >= th (column order preserved, so row-sorted columns stay sorted).
// Column sums are tree reductions (the reference sums in storage order); a decision can differ only
// when a sum lies within rounding of pct.
//
// Kernels (HBM-bound streaming over the column values; no MFMA):
//   k_mcl_stats   wave per column: nU, nP, sP, the column's mode, list of columns needing k-select
//   k_mcl_select  workgroup per listed column: radix select (8-bit digits, MSB first) of the k-th
//                 largest order-preserving key, LDS histogram, wave-parallel digit search
//   k_mcl_count   wave per column: kept entries -> scan -> colptr
//   k_mcl_compact wave per column: ballot compaction in column order
//   k_mcl_fused   (default) workgroup per column: the first three in one read of the values (LDS-staged
//                 column; both k-th values from one 10-bit histogram below the column's common key prefix,
//                 block_kth2); CBG_MCL_RADIX=1 keeps the 8-bit radix passes in the fused kernel
//                 (k_mcl_fused_radix), CBG_MCL_SPLIT=1 runs the three kernels instead.
//                 (A wave-per-column variant holding the column in registers was measured slower: 436 VGPRs,
//                 one wave per SIMD -- profiles/r03i_config4_prune_variants.txt.)
#include "spgemm_host.hpp"

namespace cbg {
namespace {

template <typename V> struct KeyOf;
template <> struct KeyOf<double> {
  using K = unsigned long long;
  static __device__ __forceinline__ K key(double v) {
    K b = (K)__double_as_longlong(v);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
  }
  static __device__ __forceinline__ double val(K k) {
    K b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
    return __longlong_as_double((long long)b);
  }
};
template <> struct KeyOf<float> {
  using K = unsigned int;
  static __device__ __forceinline__ K key(float v) {
    K b = (K)__float_as_uint(v);
    return (b >> 31) ? ~b : (b | 0x80000000u);
  }
  static __device__ __forceinline__ float val(K k) {
    K b = (k >> 31) ? (k & 0x7fffffffu) : ~k;
    return __uint_as_float(b);
  }
};

template <typename V> __device__ __forceinline__ V vmin_pos();
template <> __device__ __forceinline__ double vmin_pos<double>() { return 2.2250738585072014e-308; }
template <> __device__ __forceinline__ float vmin_pos<float>() { return 1.17549435e-38f; }

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, kWave);
  return v;
}

enum { kModeThr = 0, kModeRecover = 1, kModeSelect = 2 };

struct MclParams {
  double thr, pct;
  int64_t S, R;
};

template <typename V>
__global__ void __launch_bounds__(256) k_mcl_stats(int64_t ncol, const int64_t* __restrict__ cp,
                                                   const V* __restrict__ val, MclParams p, V* __restrict__ th,
                                                   int32_t* __restrict__ mode, int32_t* __restrict__ list,
                                                   unsigned long long* __restrict__ counters) {
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t j = (int64_t)blockIdx.x * 4 + threadIdx.x / kWave; j < ncol; j += nw) {
    const int64_t a = cp[j], b = cp[j + 1];
    const V thr = (V)p.thr;
    int64_t np = 0;
    V sp = 0;
    for (int64_t k = a + lane_id(); k < b; k += kWave) {
      const V v = val[k];
      if (v > thr) { ++np; sp += v; }
    }
    np = wave_sum(np);
    sp = wave_sum(sp);
    if (lane_id() == 0) {
      const int64_t nu = b - a;
      int m = kModeThr;
      if (np < p.R && nu > np && sp < (V)p.pct) m = kModeRecover;
      else if (p.S > 0 && np > p.S) m = kModeSelect;
      mode[j] = m;
      th[j] = thr;
      if (m != kModeThr) {
        const unsigned long long slot = atomicAdd(&counters[0], 1ull);
        list[slot] = (int32_t)j;
        atomicAdd(&counters[m], 1ull);
      }
    }
  }
}

// k-th largest value of the n values ld(0..n-1) (Kselect1 semantics); all NT threads of the block call it
template <typename V, int NT, class LD>
__device__ V block_kth_ld(LD ld, int64_t n, int64_t k, unsigned* hist, V* red, unsigned long long* bc) {
  using KO = KeyOf<V>;
  using K = typename KO::K;
  constexpr int B = 8 * (int)sizeof(K);
  if (n == 0) return vmin_pos<V>();
  if (n < k) {   // fewer than k entries: the smallest one (last of the descending partial sort)
    V m = ld(0);
    for (int64_t i = threadIdx.x; i < n; i += NT) m = min(m, ld(i));
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) m = min(m, __shfl_xor(m, d, kWave));
    if (lane_id() == 0) red[threadIdx.x / kWave] = m;
    __syncthreads();
    V r = red[0];
    for (int w = 1; w < NT / kWave; ++w) r = min(r, red[w]);
    __syncthreads();
    return r;
  }
  K prefix = 0;
  int64_t kr = k;
  for (int shift = B - 8; shift >= 0; shift -= 8) {
    for (int i = threadIdx.x; i < 256; i += NT) hist[i] = 0;
    __syncthreads();
    const K himask = (shift + 8 >= B) ? (K)0 : ~(((K)1 << (shift + 8)) - 1);
    for (int64_t i = threadIdx.x; i < n; i += NT) {
      const K key = KO::key(ld(i));
      if ((key & himask) == prefix) atomicAdd(&hist[(key >> shift) & 255], 1u);
    }
    __syncthreads();
    if (threadIdx.x < kWave) {   // wave 0: suffix sums over digits 255..0, lane l owns digits 4l..4l+3
      const int l = threadIdx.x;
      const unsigned h0 = hist[4 * l], h1 = hist[4 * l + 1], h2 = hist[4 * l + 2], h3 = hist[4 * l + 3];
      const unsigned own = h0 + h1 + h2 + h3;
      unsigned incl = own;   // inclusive suffix over lanes >= l
#pragma unroll
      for (int d = 1; d < kWave; d <<= 1) {
        const unsigned t = __shfl_down(incl, d, kWave);
        if (l + d < kWave) incl += t;
      }
      const unsigned above = incl - own;   // entries in digits > 4l+3
      if ((int64_t)above < kr && (int64_t)incl >= kr) {   // exactly one lane holds the k-th
        int64_t c = (int64_t)above;
        int dig;
        if (c + h3 >= kr) dig = 4 * l + 3;
        else if ((c += h3) + h2 >= kr) dig = 4 * l + 2;
        else if ((c += h2) + h1 >= kr) dig = 4 * l + 1;
        else { c += h1; dig = 4 * l; }
        bc[0] = (unsigned long long)dig;
        bc[1] = (unsigned long long)(kr - c);
      }
    }
    __syncthreads();
    prefix |= (K)bc[0] << shift;
    kr = (int64_t)bc[1];
    __syncthreads();
  }
  return KO::val(prefix);
}

template <typename V, int NT>
__device__ V block_kth(const V* __restrict__ val, int64_t a, int64_t b, int64_t k, unsigned* hist, V* red,
                       unsigned long long* bc) {
  return block_kth_ld<V, NT>([&](int64_t i) { return val[a + i]; }, b - a, k, hist, red, bc);
}

// Both k-th largest values of one column from ONE histogram (k_mcl_fused's selection): the keys' common
// prefix comes from the column's key range (kmin..kmax, taken in the statistics pass), one kSelBits-bit digit
// below it buckets the column, a block suffix scan finds the bucket of each target, the (few) keys of those
// buckets are gathered into LDS lists and wave q ranks list q exactly.  Six barriers instead of block_kth's
// four per 8-bit digit; a list that overflows kSelList falls back to block_kth_ld for that target.
// Preconditions: 1 <= k0 <= n; k1 == 0 (no second target) or 1 <= k1 <= n.
constexpr int kSelBits = 10, kSelBins = 1 << kSelBits, kSelList = 128;

template <typename K> struct SelScratch {
  unsigned hist[kSelBins];
  K list[2][kSelList];
  unsigned lcnt[2], wtot[8];
  int dig[2];
  int64_t kr[2];
  K res[2];
};

template <typename V, int NT, class LD>
__device__ void block_kth2(LD ld, int64_t n, int64_t k0, int64_t k1, typename KeyOf<V>::K kmin,
                           typename KeyOf<V>::K kmax, SelScratch<typename KeyOf<V>::K>& s, V* red,
                           unsigned long long* bc, V& t0, V& t1) {
  using KO = KeyOf<V>;
  using K = typename KO::K;
  constexpr int B = 8 * (int)sizeof(K);
  constexpr int PB = kSelBins / NT;   // thread t owns bins PB*t .. PB*t+PB-1
  static_assert(PB * NT == kSelBins && PB >= 1 && NT / kWave <= 8, "bins split evenly over the threads");
  if (kmin == kmax) { t0 = t1 = KO::val(kmax); return; }
  const K dx = kmin ^ kmax;
  const int vb = B - (sizeof(K) == 8 ? __builtin_clzll((unsigned long long)dx) : __builtin_clz((unsigned)dx));
  const int shift = vb > kSelBits ? vb - kSelBits : 0;
  const int tid = threadIdx.x, w = tid / kWave, l = lane_id();
  for (int i = tid; i < kSelBins; i += NT) s.hist[i] = 0;
  if (tid < 2) s.lcnt[tid] = 0;
  __syncthreads();
  for (int64_t i = tid; i < n; i += NT) atomicAdd(&s.hist[(KO::key(ld(i)) >> shift) & (kSelBins - 1)], 1u);
  __syncthreads();
  unsigned h[PB], own = 0;
#pragma unroll
  for (int u = 0; u < PB; ++u) { h[u] = s.hist[PB * tid + u]; own += h[u]; }
  unsigned incl = own;   // inclusive suffix over the wave's lanes >= l
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const unsigned t = __shfl_down(incl, d, kWave);
    if (l + d < kWave) incl += t;
  }
  if (l == 0) s.wtot[w] = incl;
  __syncthreads();
  for (int v = w + 1; v < NT / kWave; ++v) incl += s.wtot[v];
  const unsigned above = incl - own;   // entries in bins > PB*t+PB-1
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int64_t kq = q ? k1 : k0;
    if (kq > 0 && (int64_t)above < kq && (int64_t)incl >= kq) {   // exactly one thread holds target q
      int64_t c = (int64_t)above;
      int dg = PB * tid;
#pragma unroll
      for (int u = PB - 1; u >= 0; --u) {   // highest bin first: the k-th largest
        if (c + h[u] >= kq) { dg = PB * tid + u; break; }
        c += h[u];
      }
      s.dig[q] = dg;
      s.kr[q] = kq - c;
    }
  }
  __syncthreads();
  const int d0 = s.dig[0], d1 = k1 > 0 ? s.dig[1] : -1;
  for (int64_t i = tid; i < n; i += NT) {
    const K key = KO::key(ld(i));
    const int dg = (int)((key >> shift) & (kSelBins - 1));
    if (dg == d0) { const unsigned at = atomicAdd(&s.lcnt[0], 1u); if (at < kSelList) s.list[0][at] = key; }
    if (dg == d1) { const unsigned at = atomicAdd(&s.lcnt[1], 1u); if (at < kSelList) s.list[1][at] = key; }
  }
  __syncthreads();
  if (w < 2 && (w == 0 || k1 > 0)) {   // wave q ranks list q: the key with gt < kr <= ge is the answer
    const unsigned m = s.lcnt[w];
    if (m <= (unsigned)kSelList) {
      const int64_t kr = s.kr[w];
#pragma unroll
      for (int h = 0; h < kSelList / kWave; ++h) {
        const unsigned e = l + h * kWave;
        if (e < m) {
          const K x = s.list[w][e];
          int64_t gt = 0, ge = 0;
          for (unsigned y = 0; y < m; ++y) {
            const K z = s.list[w][y];
            gt += z > x;
            ge += z >= x;
          }
          if (gt < kr && ge >= kr) s.res[w] = x;   // equal keys write the same value
        }
      }
    }
  }
  __syncthreads();
  const bool of0 = s.lcnt[0] > (unsigned)kSelList, of1 = k1 > 0 && s.lcnt[1] > (unsigned)kSelList;
  t0 = KO::val(s.res[0]);
  t1 = k1 > 0 ? KO::val(s.res[1]) : V(0);
  __syncthreads();
  if (of0) t0 = block_kth_ld<V, NT>(ld, n, k0, s.hist, red, bc);
  if (of1) t1 = block_kth_ld<V, NT>(ld, n, k1, s.hist, red, bc);
}

// One pass over the column values for everything but the compaction: the column is staged in LDS (columns of
// up to kMclCap entries; longer ones are read from HBM), all waves take the statistics (nP, sP, the kept count at
// thr and the key range), block_kth2 finds the select and the recover targets from one histogram, and one more
// pass gives the recovery-after-selection test and the kept count for both candidate thresholds -- one read of
// the values instead of k_mcl_stats + k_mcl_select + k_mcl_count's three.  (k_mcl_fused_radix, behind
// CBG_MCL_RADIX=1, is the same kernel with k_mcl_select's 8-bit radix passes and wave-0 statistics.)
constexpr int kMclCap = 4096;

template <typename V, int NT>
__device__ __forceinline__ void stage_column(V* lv, const V* __restrict__ val, int64_t a, int64_t n) {
  for (int64_t i0 = threadIdx.x; i0 < n; i0 += 8 * NT) {   // 8 independent loads in flight, then the stores
    V r[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) r[u] = i0 + u * NT < n ? val[a + i0 + u * NT] : V(0);
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (i0 + u * NT < n) lv[i0 + u * NT] = r[u];
  }
}

template <typename V, int NT, int CAP>
__global__ void __launch_bounds__(NT) k_mcl_fused(int64_t ncol, const int64_t* __restrict__ cp,
                                                  const V* __restrict__ val, MclParams p, V* __restrict__ th,
                                                  int64_t* __restrict__ cnt, unsigned long long* __restrict__ counters) {
  using KO = KeyOf<V>;
  using K = typename KO::K;
  constexpr int NW = NT / kWave;
  __shared__ V lv[CAP];
  __shared__ SelScratch<K> ss;
  __shared__ V red[NW], wsp[NW];
  __shared__ int64_t wnp[NW], wge[NW], wn1[NW], wnr[NW];   // second-pass sums in their own slots: no barrier
  __shared__ K wkmn[NW], wkmx[NW];
  __shared__ unsigned long long bc[2];
  const int w = threadIdx.x / kWave;
  for (int64_t j = blockIdx.x; j < ncol; j += gridDim.x) {
    const int64_t a = cp[j], b = cp[j + 1], n = b - a;
    const bool inl = n <= CAP;
    if (inl) stage_column<V, NT>(lv, val, a, n);
    __syncthreads();
    auto ld = [&](int64_t i) -> V { return inl ? lv[i] : val[a + i]; };
    const V thr = (V)p.thr;
    {   // column statistics over all waves: nP = |v > thr|, sP, |v >= thr| (the kept count at thr), key range
      int64_t np = 0, nge = 0;
      V sp = 0;
      K kmn = ~K(0), kmx = 0;
      for (int64_t i = threadIdx.x; i < n; i += NT) {
        const V v = ld(i);
        if (v > thr) { ++np; sp += v; }
        nge += v >= thr;
        const K key = KO::key(v);
        kmn = min(kmn, key);
        kmx = max(kmx, key);
      }
      np = wave_sum(np);
      nge = wave_sum(nge);
      sp = wave_sum(sp);
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) {
        kmn = min(kmn, (K)__shfl_xor(kmn, d, kWave));
        kmx = max(kmx, (K)__shfl_xor(kmx, d, kWave));
      }
      if (lane_id() == 0) { wnp[w] = np; wge[w] = nge; wsp[w] = sp; wkmn[w] = kmn; wkmx[w] = kmx; }
    }
    __syncthreads();
    int64_t NP = 0, C = 0;
    V SP = 0;
    K kmn = ~K(0), kmx = 0;
    for (int v = 0; v < NW; ++v) {
      NP += wnp[v]; C += wge[v]; SP += wsp[v];
      kmn = min(kmn, wkmn[v]);
      kmx = max(kmx, wkmx[v]);
    }
    int m = kModeThr;
    if (NP < p.R && n > NP && SP < (V)p.pct) m = kModeRecover;
    else if (p.S > 0 && NP > p.S) m = kModeSelect;
    if (threadIdx.x == 0 && m != kModeThr) atomicAdd(&counters[m], 1ull);
    V t = thr;
    if (m != kModeThr) {
      // Kselect1 targets: kth(S) for select, kth(R) for recover or recovery after selection; k > n -> the
      // column minimum (n >= 1 here: nP > S >= 1 or nU > nP)
      const V vmin = KO::val(kmn);
      const int64_t kR = p.R > 0 && p.R <= n ? p.R : 0;
      V r0 = vmin, r1 = vmin;
      if (m == kModeSelect) block_kth2<V, NT>(ld, n, p.S, kR, kmn, kmx, ss, red, bc, r0, r1);   // S < nP <= n
      else if (kR > 0) block_kth2<V, NT>(ld, n, kR, 0, kmn, kmx, ss, red, bc, r1, r0);
      const V tS = r0, tR = r1;
      // one pass: the kept count at the final threshold, and for selection the recovery test
      // (ParFriends.h:290-333: n1 = |v >= tS|, s1 = sum{v >= tS}; n1 < R && s1 < pct -> tR)
      const bool sel = m == kModeSelect;
      int64_t n1 = 0, nr = 0;
      V s1 = 0;
      for (int64_t i = threadIdx.x; i < n; i += NT) {
        const V v = ld(i);
        if (sel && v >= tS) { ++n1; s1 += v; }
        nr += v >= tR;
      }
      n1 = wave_sum(n1);
      nr = wave_sum(nr);
      s1 = wave_sum(s1);
      if (lane_id() == 0) { wn1[w] = n1; wnr[w] = nr; red[w] = s1; }
      __syncthreads();
      int64_t N1 = 0, NR = 0;
      V S1 = 0;
      for (int v = 0; v < NW; ++v) { N1 += wn1[v]; NR += wnr[v]; S1 += red[v]; }
      if (!sel) {
        t = tR; C = NR;
      } else if (p.R > 0 && N1 < p.R && S1 < (V)p.pct) {
        t = tR; C = NR;
        if (threadIdx.x == 0) atomicAdd(&counters[3], 1ull);
      } else {
        t = tS; C = N1;
      }
    }
    if (threadIdx.x == 0) { cnt[j] = C; th[j] = t; }
    __syncthreads();
  }
}

template <typename V, int NT>
__global__ void __launch_bounds__(NT) k_mcl_fused_radix(int64_t ncol, const int64_t* __restrict__ cp,
                                                        const V* __restrict__ val, MclParams p, V* __restrict__ th,
                                                        int64_t* __restrict__ cnt,
                                                        unsigned long long* __restrict__ counters) {
  __shared__ V lv[kMclCap];
  __shared__ unsigned hist[256];
  __shared__ V red[NT / kWave];
  __shared__ int64_t rn[NT / kWave];
  __shared__ unsigned long long bc[2];
  __shared__ int smode;
  for (int64_t j = blockIdx.x; j < ncol; j += gridDim.x) {
    const int64_t a = cp[j], b = cp[j + 1], n = b - a;
    const bool inl = n <= kMclCap;
    if (inl) stage_column<V, NT>(lv, val, a, n);
    __syncthreads();
    auto ld = [&](int64_t i) -> V { return inl ? lv[i] : val[a + i]; };
    const V thr = (V)p.thr;
    if (threadIdx.x < kWave) {   // column statistics, in k_mcl_stats' lane order
      int64_t np = 0;
      V sp = 0;
      for (int64_t k = lane_id(); k < n; k += kWave) {
        const V v = ld(k);
        if (v > thr) { ++np; sp += v; }
      }
      np = wave_sum(np);
      sp = wave_sum(sp);
      if (lane_id() == 0) {
        int m = kModeThr;
        if (np < p.R && n > np && sp < (V)p.pct) m = kModeRecover;
        else if (p.S > 0 && np > p.S) m = kModeSelect;
        smode = m;
        if (m != kModeThr) atomicAdd(&counters[m], 1ull);
      }
    }
    __syncthreads();
    const int m = smode;
    V t = thr;
    if (m == kModeRecover) {
      t = block_kth_ld<V, NT>(ld, n, p.R, hist, red, bc);
    } else if (m == kModeSelect) {
      t = block_kth_ld<V, NT>(ld, n, p.S, hist, red, bc);
      if (p.R > 0) {   // recovery after selection (ParFriends.h:290-333), k_mcl_select's order
        int64_t n1 = 0;
        V s1 = 0;
        for (int64_t i = threadIdx.x; i < n; i += NT) {
          const V v = ld(i);
          if (v >= t) { ++n1; s1 += v; }
        }
        n1 = wave_sum(n1);
        s1 = wave_sum(s1);
        if (lane_id() == 0) { rn[threadIdx.x / kWave] = n1; red[threadIdx.x / kWave] = s1; }
        __syncthreads();
        int64_t N1 = 0;
        V S1 = 0;
        for (int w = 0; w < NT / kWave; ++w) { N1 += rn[w]; S1 += red[w]; }
        __syncthreads();
        if (N1 < p.R && S1 < (V)p.pct) {
          t = block_kth_ld<V, NT>(ld, n, p.R, hist, red, bc);
          if (threadIdx.x == 0) atomicAdd(&counters[3], 1ull);
        }
      }
    }
    int64_t c = 0;   // kept entries (v >= t)
    for (int64_t i = threadIdx.x; i < n; i += NT) c += ld(i) >= t;
    c = wave_sum(c);
    if (lane_id() == 0) rn[threadIdx.x / kWave] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
      int64_t C = 0;
      for (int w = 0; w < NT / kWave; ++w) C += rn[w];
      cnt[j] = C;
      th[j] = t;
    }
    __syncthreads();
  }
}

template <typename V, int NT>
__global__ void __launch_bounds__(NT) k_mcl_select(const int32_t* __restrict__ list,
                                                   const unsigned long long* __restrict__ count,
                                                   const int64_t* __restrict__ cp, const V* __restrict__ val,
                                                   MclParams p, V* __restrict__ th, const int32_t* __restrict__ mode,
                                                   unsigned long long* __restrict__ counters) {
  __shared__ unsigned hist[256];
  __shared__ V red[NT / kWave];
  __shared__ int64_t rn[NT / kWave];
  __shared__ unsigned long long bc[2];
  const int64_t n = (int64_t)count[0];
  for (int64_t it = blockIdx.x; it < n; it += gridDim.x) {
    const int32_t j = list[it];
    const int64_t a = cp[j], b = cp[j + 1];
    const int m = mode[j];
    V t;
    if (m == kModeRecover) {
      t = block_kth<V, NT>(val, a, b, p.R, hist, red, bc);
    } else {
      t = block_kth<V, NT>(val, a, b, p.S, hist, red, bc);
      if (p.R > 0) {   // recovery after selection (ParFriends.h:290-333)
        int64_t n1 = 0;
        V s1 = 0;
        for (int64_t i = a + threadIdx.x; i < b; i += NT) {
          const V v = val[i];
          if (v >= t) { ++n1; s1 += v; }
        }
        n1 = wave_sum(n1);
        s1 = wave_sum(s1);
        if (lane_id() == 0) { rn[threadIdx.x / kWave] = n1; red[threadIdx.x / kWave] = s1; }
        __syncthreads();
        int64_t N1 = 0;
        V S1 = 0;
        for (int w = 0; w < NT / kWave; ++w) { N1 += rn[w]; S1 += red[w]; }
        __syncthreads();
        if (N1 < p.R && S1 < (V)p.pct) {
          t = block_kth<V, NT>(val, a, b, p.R, hist, red, bc);
          if (threadIdx.x == 0) atomicAdd(&counters[3], 1ull);
        }
      }
    }
    if (threadIdx.x == 0) th[j] = t;
    __syncthreads();
  }
}

template <typename V>
__global__ void __launch_bounds__(256) k_mcl_count(int64_t ncol, const int64_t* __restrict__ cp,
                                                   const V* __restrict__ val, const V* __restrict__ th,
                                                   int64_t* __restrict__ cnt) {
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t j = (int64_t)blockIdx.x * 4 + threadIdx.x / kWave; j < ncol; j += nw) {
    const int64_t a = cp[j], b = cp[j + 1];
    const V t = th[j];
    int64_t c = 0;
    for (int64_t k = a + lane_id(); k < b; k += kWave) c += val[k] >= t;
    c = wave_sum(c);
    if (lane_id() == 0) cnt[j] = c;
  }
}

template <typename V>
__global__ void __launch_bounds__(256) k_mcl_compact(int64_t ncol, const int64_t* __restrict__ cp,
                                                     const int32_t* __restrict__ ir, const V* __restrict__ val,
                                                     const V* __restrict__ th, const int64_t* __restrict__ ocp,
                                                     int32_t* __restrict__ oir, V* __restrict__ oval) {
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int l = lane_id();
  const unsigned long long below = (1ull << l) - 1ull;
  for (int64_t j = (int64_t)blockIdx.x * 4 + threadIdx.x / kWave; j < ncol; j += nw) {
    const int64_t a = cp[j], b = cp[j + 1];
    const V t = th[j];
    int64_t o = ocp[j];
    for (int64_t k0 = a; k0 < b; k0 += 4 * kWave) {   // four chunks' loads in flight, then their compaction
      V v[4];
      int32_t r[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t k = k0 + u * kWave + l;
        v[u] = k < b ? val[k] : V(0);
        r[u] = k < b ? ir[k] : 0;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bool keep = k0 + u * kWave + l < b && v[u] >= t;
        const unsigned long long m = __ballot(keep);
        if (keep) {
          const int64_t d = o + __popcll(m & below);
          oir[d] = r[u];
          oval[d] = v[u];
        }
        o += __popcll(m);
      }
    }
  }
}

// rebased column range [c0, c1) of a CSC: colptr - cp[c0]
__global__ void k_col_rebase(int64_t n, const int64_t* __restrict__ cp, int64_t c0, int64_t* __restrict__ out) {
  const int64_t base = cp[c0];
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i <= n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = cp[c0 + i] - base;
}
// column subset: cnt[i] = nnz of column cols[i]
__global__ void k_sel_count(int64_t n, const int64_t* __restrict__ cp, const int64_t* __restrict__ cols,
                            int64_t* __restrict__ cnt) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    cnt[i] = cp[cols[i] + 1] - cp[cols[i]];
}
// one wavefront per selected column copies its rows and values
template <typename T>
__global__ void __launch_bounds__(256) k_sel_copy(int64_t n, const int64_t* __restrict__ cp,
                                                  const int32_t* __restrict__ ir, const T* __restrict__ val,
                                                  const int64_t* __restrict__ cols, const int64_t* __restrict__ ocp,
                                                  int32_t* __restrict__ oir, T* __restrict__ oval) {
  const int w = threadIdx.x / kWave, l = lane_id();
  for (int64_t i = blockIdx.x * 4 + w; i < n; i += (int64_t)gridDim.x * 4) {
    const int64_t s = cp[cols[i]], len = cp[cols[i] + 1] - s, o = ocp[i];
    for (int64_t e = l; e < len; e += kWave) {
      oir[o + e] = ir[s + e];
      if (val) oval[o + e] = val[s + e];
    }
  }
}
// colptr of part q appended at column offset `coff` and entry offset `eoff`
__global__ void k_col_shift(int64_t n, const int64_t* __restrict__ cp, int64_t eoff, int64_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i <= n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = cp[i] + eoff;
}

}  // namespace
}  // namespace cbg

namespace {
template <typename V>
cbg_status mcl_prune_impl(cbg_ctx* ctx, const cbg_csc_result* in, const MclParams& p, cbg_csc_result* out,
                          cbg_mcl_stats* stats) {
  hipStream_t st = ctx->stream;
  const int64_t N = in->ncol, nnz = in->nnz;
  std::unique_ptr<Owner> own(new Owner(ctx->pool));
  HIPCHK(own->cp.reserve(sizeof(int64_t) * (N + 1)));
  PoolBuf th, mode, list, cnt, tiles;
  for (PoolBuf* b : {&th, &mode, &list, &cnt, &tiles}) b->pool = ctx->pool;
  HIPCHK(th.reserve(sizeof(V) * (N + 1)));
  HIPCHK(mode.reserve(sizeof(int32_t) * (N + 1)));
  HIPCHK(list.reserve(sizeof(int32_t) * (N + 1)));
  HIPCHK(cnt.reserve(sizeof(int64_t) * (N + 1)));
  HIPCHK(ctx->scalars.reserve(256));
  unsigned long long* sc = ctx->scalars.as<unsigned long long>();
  HIPCHK(hipMemsetAsync(sc, 0, 64, st));
  const V* val = (const V*)in->val;
  const int gw = (int)grid_for(N, 4, kMaxGrid * 2);
  static const bool split_passes = [] { const char* e = std::getenv("CBG_MCL_SPLIT"); return e && e[0] == '1'; }();
  if (N > 0 && split_passes) {   // the three-pass form (stats, select of the listed columns, count)
    k_mcl_stats<V><<<gw, 256, 0, st>>>(N, in->colptr, val, p, th.as<V>(), mode.as<int32_t>(), list.as<int32_t>(), sc);
    k_mcl_select<V, 256><<<(int)grid_for(N, 1, kMaxGrid * 2), 256, 0, st>>>(
        list.as<int32_t>(), sc, in->colptr, val, p, th.as<V>(), mode.as<int32_t>(), sc);
    k_mcl_count<V><<<gw, 256, 0, st>>>(N, in->colptr, val, th.as<V>(), cnt.as<int64_t>());
  } else if (N > 0) {
    static const bool radix = [] { const char* e = std::getenv("CBG_MCL_RADIX"); return e && e[0] == '1'; }();
    const int g = (int)grid_for(N, 1, kMaxGrid * 8);
    if (radix)
      k_mcl_fused_radix<V, 256><<<g, 256, 0, st>>>(N, in->colptr, val, p, th.as<V>(), cnt.as<int64_t>(), sc);
    else
      k_mcl_fused<V, 256, kMclCap><<<g, 256, 0, st>>>(N, in->colptr, val, p, th.as<V>(), cnt.as<int64_t>(), sc);
  }
  if (N > 0) {
    const int64_t ntiles = (N + kScanTile - 1) / kScanTile;
    HIPCHK(tiles.reserve(sizeof(int64_t) * (ntiles + 1)));
    k_scan_tiles<<<(int)ntiles, 256, 0, st>>>(N, cnt.as<int64_t>(), tiles.as<int64_t>());
    k_scan_sums<<<1, 1024, 0, st>>>(ntiles, tiles.as<int64_t>(), (int64_t*)(sc + 4));
    k_scan_apply<<<(int)ntiles, 256, 0, st>>>(N, cnt.as<int64_t>(), tiles.as<int64_t>(), own->cp.as<int64_t>());
  } else {
    HIPCHK(hipMemsetAsync(own->cp.p, 0, sizeof(int64_t), st));
  }
  HIPCHK(hipGetLastError());
  unsigned long long h[8] = {};
  HIPCHK(hipMemcpyAsync(h, sc, 64, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  const int64_t onnz = N > 0 ? (int64_t)h[4] : 0;
  HIPCHK(own->ir.reserve(sizeof(int32_t) * (onnz + 1)));
  HIPCHK(own->val.reserve(sizeof(V) * (onnz + 1)));
  if (N > 0 && nnz > 0)
    k_mcl_compact<V><<<gw, 256, 0, st>>>(N, in->colptr, in->row, val, th.as<V>(), own->cp.as<int64_t>(),
                                         own->ir.as<int32_t>(), own->val.as<V>());
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(st));   // th/mode/list/cnt go back to the pool on return
  memset(out, 0, sizeof(*out));
  out->nrow = in->nrow; out->ncol = N; out->nnz = onnz;
  out->colptr = own->cp.as<int64_t>(); out->row = own->ir.as<int32_t>(); out->val = own->val.p;
  out->val_type = in->val_type; out->multiplies = in->multiplies;
  out->_owner = own.release();
  if (stats) {
    stats->recovered = (int64_t)h[kModeRecover];
    stats->selected = (int64_t)h[kModeSelect];
    stats->recovered_after_select = (int64_t)h[3];
    stats->nnz_in = nnz;
    stats->nnz_out = onnz;
  }
  return CBG_OK;
}
}  // namespace

extern "C" cbg_status cbg_mcl_prune(cbg_ctx* ctx, const cbg_csc_result* in, double hardThreshold, int64_t selectNum,
                                    int64_t recoverNum, double recoverPct, cbg_csc_result* out,
                                    cbg_mcl_stats* stats) {
  if (!ctx || !in || !out) return CBG_EINVAL;
  if (in->nnz > 0 && (!in->row || !in->val)) return CBG_EINVAL;
  HIPCHK(hipSetDevice(ctx->device));
  MclParams p{hardThreshold, recoverPct, selectNum, recoverNum};
  if (in->val_type == CBG_F64) return mcl_prune_impl<double>(ctx, in, p, out, stats);
  if (in->val_type == CBG_F32) return mcl_prune_impl<float>(ctx, in, p, out, stats);
  return CBG_EUNSUP;
}

extern "C" cbg_status cbg_col_range(cbg_ctx* ctx, const cbg_csc_result* in, int64_t c0, int64_t c1,
                                    cbg_csc_result* out) {
  if (!ctx || !in || !out) return CBG_EINVAL;
  if (c0 < 0 || c1 < c0 || c1 > in->ncol) return CBG_EDIM;
  HIPCHK(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  int64_t e[2];
  HIPCHK(hipMemcpyAsync(&e[0], in->colptr + c0, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(&e[1], in->colptr + c1, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  const int64_t n = c1 - c0, nnz = e[1] - e[0];
  const size_t vs = in->val ? dt_size(in->val_type) : 0;
  std::unique_ptr<Owner> own(new Owner(ctx->pool));
  HIPCHK(own->cp.reserve(sizeof(int64_t) * (n + 1)));
  HIPCHK(own->ir.reserve(sizeof(int32_t) * (nnz + 1)));
  HIPCHK(own->val.reserve(vs * (nnz + 1) + 8));
  k_col_rebase<<<(int)grid_for(n + 1, 256, kMaxGrid), 256, 0, st>>>(n, in->colptr, c0, own->cp.as<int64_t>());
  if (nnz) HIPCHK(hipMemcpyAsync(own->ir.p, in->row + e[0], 4 * nnz, hipMemcpyDeviceToDevice, st));
  if (nnz && vs) HIPCHK(hipMemcpyAsync(own->val.p, (const char*)in->val + vs * e[0], vs * nnz, hipMemcpyDeviceToDevice, st));
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(st));
  memset(out, 0, sizeof(*out));
  out->nrow = in->nrow; out->ncol = n; out->nnz = nnz;
  out->colptr = own->cp.as<int64_t>(); out->row = own->ir.as<int32_t>(); out->val = vs ? own->val.p : nullptr;
  out->val_type = in->val_type;
  out->_owner = own.release();
  return CBG_OK;
}

extern "C" cbg_status cbg_col_select(cbg_ctx* ctx, const cbg_csc_result* in, const int64_t* cols, int64_t ncols,
                                     cbg_csc_result* out) {
  if (!ctx || !in || !out || (ncols > 0 && !cols) || ncols < 0) return CBG_EINVAL;
  for (int64_t i = 0; i < ncols; ++i)
    if (cols[i] < 0 || cols[i] >= in->ncol) return CBG_EDIM;
  HIPCHK(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  const size_t vs = in->val ? dt_size(in->val_type) : 0;
  std::unique_ptr<Owner> own(new Owner(ctx->pool));
  HIPCHK(own->cp.reserve(sizeof(int64_t) * (ncols + 1)));
  PoolBuf dcols, cnt, tiles;
  for (PoolBuf* b : {&dcols, &cnt, &tiles}) b->pool = ctx->pool;
  HIPCHK(dcols.reserve(sizeof(int64_t) * (ncols + 1)));
  HIPCHK(cnt.reserve(sizeof(int64_t) * (ncols + 1)));
  HIPCHK(ctx->scalars.reserve(256));
  int64_t nnz = 0;
  if (ncols > 0) {
    HIPCHK(hipMemcpyAsync(dcols.p, cols, sizeof(int64_t) * ncols, hipMemcpyHostToDevice, st));
    k_sel_count<<<(int)grid_for(ncols, 256, kMaxGrid), 256, 0, st>>>(ncols, in->colptr, dcols.as<int64_t>(),
                                                                     cnt.as<int64_t>());
    const int64_t ntiles = (ncols + kScanTile - 1) / kScanTile;
    HIPCHK(tiles.reserve(sizeof(int64_t) * (ntiles + 1)));
    int64_t* tot = (int64_t*)ctx->scalars.p;
    k_scan_tiles<<<(int)ntiles, 256, 0, st>>>(ncols, cnt.as<int64_t>(), tiles.as<int64_t>());
    k_scan_sums<<<1, 1024, 0, st>>>(ntiles, tiles.as<int64_t>(), tot);
    k_scan_apply<<<(int)ntiles, 256, 0, st>>>(ncols, cnt.as<int64_t>(), tiles.as<int64_t>(), own->cp.as<int64_t>());
    HIPCHK(hipMemcpyAsync(&nnz, tot, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  } else {
    HIPCHK(hipMemsetAsync(own->cp.p, 0, sizeof(int64_t), st));
  }
  HIPCHK(own->ir.reserve(sizeof(int32_t) * (nnz + 1)));
  HIPCHK(own->val.reserve(vs * (nnz + 1) + 8));
  if (nnz > 0) {
    const int g = (int)grid_for(ncols, 4, kMaxGrid * 2);
    const int64_t* c = dcols.as<int64_t>();
    int64_t* ocp = own->cp.as<int64_t>();
    int32_t* oir = own->ir.as<int32_t>();
    switch (vs) {
      case 1: k_sel_copy<uint8_t><<<g, 256, 0, st>>>(ncols, in->colptr, in->row, (const uint8_t*)in->val, c, ocp, oir, (uint8_t*)own->val.p); break;
      case 4: k_sel_copy<uint32_t><<<g, 256, 0, st>>>(ncols, in->colptr, in->row, (const uint32_t*)in->val, c, ocp, oir, (uint32_t*)own->val.p); break;
      default: k_sel_copy<uint64_t><<<g, 256, 0, st>>>(ncols, in->colptr, in->row, (const uint64_t*)in->val, c, ocp, oir, (uint64_t*)own->val.p); break;
    }
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(st));   // dcols/cnt/tiles go back to the pool on return
  memset(out, 0, sizeof(*out));
  out->nrow = in->nrow; out->ncol = ncols; out->nnz = nnz;
  out->colptr = own->cp.as<int64_t>(); out->row = own->ir.as<int32_t>(); out->val = vs ? own->val.p : nullptr;
  out->val_type = in->val_type; out->multiplies = in->multiplies;
  out->_owner = own.release();
  return CBG_OK;
}

extern "C" cbg_status cbg_col_concat(cbg_ctx* ctx, const cbg_csc_result* parts, int32_t nparts, cbg_csc_result* out) {
  if (!ctx || !parts || nparts <= 0 || !out) return CBG_EINVAL;
  int64_t N = 0, nnz = 0;
  for (int q = 0; q < nparts; ++q) {
    if (parts[q].nrow != parts[0].nrow || parts[q].val_type != parts[0].val_type ||
        (parts[q].val == nullptr) != (parts[0].val == nullptr))
      return CBG_EDIM;
    N += parts[q].ncol;
    nnz += parts[q].nnz;
  }
  HIPCHK(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  const size_t vs = parts[0].val ? dt_size(parts[0].val_type) : 0;
  std::unique_ptr<Owner> own(new Owner(ctx->pool));
  HIPCHK(own->cp.reserve(sizeof(int64_t) * (N + 1)));
  HIPCHK(own->ir.reserve(sizeof(int32_t) * (nnz + 1)));
  HIPCHK(own->val.reserve(vs * (nnz + 1) + 8));
  int64_t coff = 0, eoff = 0;
  HIPCHK(hipMemsetAsync(own->cp.p, 0, 8, st));
  for (int q = 0; q < nparts; ++q) {
    const cbg_csc_result& P = parts[q];
    if (P.ncol)   // writes colptr[coff .. coff+ncol] (entry coff rewritten with the same value)
      k_col_shift<<<(int)grid_for(P.ncol + 1, 256, kMaxGrid), 256, 0, st>>>(P.ncol, P.colptr, eoff,
                                                                           own->cp.as<int64_t>() + coff);
    if (P.nnz) HIPCHK(hipMemcpyAsync(own->ir.as<int32_t>() + eoff, P.row, 4 * P.nnz, hipMemcpyDeviceToDevice, st));
    if (P.nnz && vs)
      HIPCHK(hipMemcpyAsync((char*)own->val.p + vs * eoff, P.val, vs * P.nnz, hipMemcpyDeviceToDevice, st));
    coff += P.ncol;
    eoff += P.nnz;
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(st));
  memset(out, 0, sizeof(*out));
  out->nrow = parts[0].nrow; out->ncol = N; out->nnz = nnz;
  out->colptr = own->cp.as<int64_t>(); out->row = own->ir.as<int32_t>(); out->val = vs ? own->val.p : nullptr;
  out->val_type = parts[0].val_type;
  out->_owner = own.release();
  return CBG_OK;
}
