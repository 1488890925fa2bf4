// galerkin.hip -- the Galerkin coarse operator on the device: MIS-2 aggregation restriction and the
// fused triple product R^T A R (BASELINE config 5).
//
// Reference (3DSpGEMM/RestrictionOp.h, RestrictionOp.cpp:155-196, ReleaseTests/GalerkinNew.cpp:100-127):
//   MIS2 (RestrictionOp.h:116-196): Luby rounds on the symmetrised loop-free graph -- every candidate
//     draws a random value, a candidate whose value beats all candidates within distance 2 joins the
//     set, and it and its distance-2 neighbourhood leave the candidate set;
//   RestrictionOp (RestrictionOp.h:198-290): every vertex joins an aggregate rooted at a set vertex
//     within distance 1, else within distance 2; R(i, agg(i)) = 1 (n x nagg), RT = R^T;
//   the driver then forms R^T A and (R^T A) R with two SpGEMMs (RestrictionOp.cpp:188-196).
// Device formulation:
//   * priorities are distinct 64-bit keys: a seeded hash of the vertex id above the id itself (the
//     reference draws from its global Mersenne twister, so its aggregation is seed-specific; the
//     host restatement combblas_amd.inputs.aggregation_restriction uses these same keys);
//   * each round is two max-propagation sweeps (distance 1, then 2) and two flag sweeps over the CSC
//     graph, one thread per vertex, and one counter read by the host;
//   * R^T A R for an aggregation R (exactly one nonzero per row, any value): C(I, J) =
//     sum over i in I, j in J of R(i,I) A(i,j) R(j,J).  One workgroup per aggregate J reads the A
//     columns of J's members (R's row order), maps their rows to aggregates, sorts and sums in LDS
//     (k_rap_agg: a count pass and a fill pass; one read of nnz(A) each instead of two SpGEMMs with
//     an R^T A intermediate; deterministic summation order).
#include "spgemm_host.hpp"
#include <algorithm>
#include <numeric>
#include <random>

namespace {

__device__ __forceinline__ uint64_t mis_key(uint32_t v, uint64_t seed) {
  uint64_t z = (uint64_t)v ^ (seed * 0x9E3779B97F4A7C15ull);
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return ((z >> 32) << 32 | v) + 1;   // distinct, nonzero; vertex = (key - 1) & 0xffffffff
}

__global__ void k_mis_keys(int64_t n, uint64_t seed, uint64_t* __restrict__ key, int8_t* __restrict__ state) {
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
    key[v] = mis_key((uint32_t)v, seed);
    state[v] = 0;
  }
}

// out[v] = max(in[v], max over neighbours u of in[u]); in = masked keys (mask: state == want) or a vector
template <bool MASKED>
__global__ void k_nbr_max(int64_t n, const int64_t* __restrict__ cp, const int32_t* __restrict__ ir,
                          const uint64_t* __restrict__ in, const int8_t* __restrict__ state, int8_t want,
                          uint64_t* __restrict__ out) {
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
    uint64_t m = (!MASKED || state[v] == want) ? in[v] : 0;
    for (int64_t p = cp[v]; p < cp[v + 1]; ++p) {
      const int32_t u = ir[p];
      const uint64_t x = (!MASKED || state[u] == want) ? in[u] : 0;
      m = x > m ? x : m;
    }
    out[v] = m;
  }
}

// new set members: undecided vertices whose key is the distance-2 maximum
__global__ void k_mis_select(int64_t n, const uint64_t* __restrict__ key, const uint64_t* __restrict__ m2,
                             const int8_t* __restrict__ state, uint8_t* __restrict__ fresh) {
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x)
    fresh[v] = state[v] == 0 && key[v] == m2[v];
}

__global__ void k_nbr_or(int64_t n, const int64_t* __restrict__ cp, const int32_t* __restrict__ ir,
                         const uint8_t* __restrict__ in, uint8_t* __restrict__ out) {
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
    uint8_t f = in[v];
    for (int64_t p = cp[v]; p < cp[v + 1] && !f; ++p) f = in[ir[p]];
    out[v] = f;
  }
}

// roots <- fresh; undecided vertices within distance 2 of a fresh root are covered; count undecided
__global__ void k_mis_update(int64_t n, const uint8_t* __restrict__ fresh, const uint8_t* __restrict__ near2,
                             int8_t* __restrict__ state, unsigned long long* __restrict__ undecided) {
  unsigned long long c = 0;
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
    int8_t s = state[v];
    if (fresh[v]) s = 1;
    else if (s == 0 && near2[v]) s = 2;
    state[v] = s;
    c += s == 0;
  }
  c = wave_sum64((int64_t)c);
  if (lane_id() == 0 && c) atomicAdd(undecided, c);
}

__global__ void k_root_keys(int64_t n, const uint64_t* __restrict__ key, const int8_t* __restrict__ state,
                            uint64_t* __restrict__ rk, int64_t* __restrict__ isroot) {
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
    rk[v] = state[v] == 1 ? key[v] : 0;
    isroot[v] = state[v] == 1;
  }
}

// agg(v) = id of the highest-key root within distance 1, else within distance 2 (root ids in vertex order)
__global__ void k_assign(int64_t n, const uint64_t* __restrict__ b1, const uint64_t* __restrict__ b2,
                         const int64_t* __restrict__ rid, int32_t* __restrict__ agg, unsigned long long* __restrict__ colcnt) {
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t b = b1[v] ? b1[v] : b2[v];
    const int32_t a = b ? (int32_t)rid[(b - 1) & 0xffffffffull] : -1;
    agg[v] = a;
    if (a >= 0) atomicAdd(&colcnt[a], 1ull);
  }
}

__global__ void k_scatter_members(int64_t n, const int32_t* __restrict__ agg, unsigned long long* __restrict__ cursor,
                                  int32_t* __restrict__ rows) {
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x)
    if (agg[v] >= 0) rows[atomicAdd(&cursor[agg[v]], 1ull)] = (int32_t)v;
}

__global__ void k_rt(int64_t n, const int32_t* __restrict__ agg, int64_t* __restrict__ cp, int32_t* __restrict__ ir,
                     double* __restrict__ val) {
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v <= n; v += (int64_t)gridDim.x * blockDim.x) {
    cp[v] = v;
    if (v < n) { ir[v] = agg[v]; val[v] = 1.0; }
  }
}

// ---------------------------------------------------------------- fused R^T A R (aggregation R)
// per row i of R: its aggregate and value; rows not covered exactly once are counted as bad
__global__ void k_r_rows(int64_t nagg, const int64_t* __restrict__ rcp, const int32_t* __restrict__ rir,
                         const double* __restrict__ rval, int32_t* __restrict__ agg, double* __restrict__ rv,
                         unsigned int* __restrict__ seen) {
  for (int64_t J = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; J < nagg; J += (int64_t)gridDim.x * blockDim.x)
    for (int64_t p = rcp[J]; p < rcp[J + 1]; ++p) {
      const int32_t i = rir[p];
      agg[i] = (int32_t)J;
      rv[i] = rval ? rval[p] : 1.0;
      atomicAdd(&seen[i], 1u);
    }
}

__global__ void k_count_bad(int64_t n, const unsigned int* __restrict__ seen, unsigned long long* __restrict__ bad) {
  unsigned long long c = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    c += seen[i] != 1;
  c = wave_sum64((int64_t)c);
  if (lane_id() == 0 && c) atomicAdd(bad, c);
}

// raw layout: member p of R (entries in column order) contributes |A(:, rir[p])| entries; the exclusive
// scan of these lengths over p is each member's raw offset, and rawcp[J] = that offset at rcp[J]
__global__ void k_member_len(int64_t nnzr, const int32_t* __restrict__ rir, const int64_t* __restrict__ acp,
                             int64_t* __restrict__ len) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < nnzr; p += (int64_t)gridDim.x * blockDim.x)
    len[p] = acp[rir[p] + 1] - acp[rir[p]];
}

// One 64-lane workgroup per aggregate J: the flattened entries of its members' A columns (member p's
// entries start at moff[p]) are loaded into LDS as keys (agg(i) << 32 | position) with values
// R(i,I) A(i,j) R(j,J), bitonic-sorted, and every run of one row is summed in position order
// (deterministic); count pass -> cnt[J], fill pass -> sorted (row, value) at ccp[J].  Aggregates with
// more than kRapCapBig entries are counted in *overflow (the caller falls back to two SpGEMMs).
constexpr int kRapCap = 512, kRapCapBig = 2048, kRapMem = 64;

// CAP = kRapCap: every aggregate; one with more entries goes to olist (when given) for the CAP = kRapCapBig pass
// (list = olist, count = its length), and only an aggregate above that is counted in *overflow.
template <int CAP>
__global__ void __launch_bounds__(64) k_rap_agg(int64_t nagg, const int32_t* __restrict__ list,
                                                const unsigned long long* __restrict__ nlist,
                                                int32_t* __restrict__ olist, unsigned long long* __restrict__ nolist,
                                                const int64_t* __restrict__ rcp,
                                                const int32_t* __restrict__ rir, const int64_t* __restrict__ acp,
                                                const int32_t* __restrict__ air, const double* __restrict__ aval,
                                                const int32_t* __restrict__ agg, const double* __restrict__ rv,
                                                const int64_t* __restrict__ moff, int64_t* __restrict__ cnt,
                                                int32_t* __restrict__ trow, double* __restrict__ tval, int64_t cap,
                                                unsigned long long* __restrict__ overflow) {
  __shared__ uint64_t key[CAP];
  __shared__ double val[CAP];
  __shared__ int32_t s_mo[kRapMem + 1];   // members' entry offsets (relative to the aggregate's first entry)
  __shared__ int64_t s_q0[kRapMem];       // members' A column starts
  __shared__ double s_rvj[kRapMem];       // R(j, J)
  const int lane = threadIdx.x;
  const int64_t nj = list ? (int64_t)*nlist : nagg;
  for (int64_t i = blockIdx.x; i < nj; i += gridDim.x) {
    const int64_t J = list ? list[i] : i;
    const int64_t p0 = rcp[J], p1 = rcp[J + 1];
    const int64_t base = moff[p0];
    const int t = (int)min<int64_t>(moff[p1] - base, CAP + 1);
    if (t > CAP || base + t > cap) {   // uniform; past `cap` only for an R that is no aggregation
      if (lane == 0) {
        cnt[J] = 0;
        if (olist && base + t <= cap) olist[atomicAdd(nolist, 1ull)] = (int32_t)J;
        else atomicAdd(overflow, 1ull);
      }
      continue;
    }
    int N = 64;
    while (N < t) N <<= 1;
    const int64_t nm = p1 - p0;
    if (nm <= kRapMem) {   // members staged: one level of member loads, then the entry -> member search in LDS
      for (int64_t m = lane; m < nm; m += 64) {
        const int32_t j = rir[p0 + m];
        s_mo[m] = (int32_t)(moff[p0 + m] - base);
        s_q0[m] = acp[j];
        s_rvj[m] = rv[j];
      }
      __syncthreads();
      for (int e = lane; e < N; e += 64) {
        if (e < t) {
          int lo = 0, hi = (int)nm - 1;   // last member m with s_mo[m] <= e
          while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (s_mo[mid] <= e) lo = mid; else hi = mid - 1;
          }
          const int64_t q = s_q0[lo] + (e - s_mo[lo]);
          const int32_t i = air[q];
          key[e] = ((uint64_t)(uint32_t)agg[i] << 32) | (uint32_t)e;
          val[e] = rv[i] * (aval ? aval[q] : 1.0) * s_rvj[lo];
        } else {
          key[e] = ~0ull;
        }
      }
    } else for (int e = lane; e < N; e += 64) {
      if (e < t) {
        int64_t lo = p0, hi = p1 - 1;   // the member holding entry e: last p with moff[p] - base <= e
        while (lo < hi) {
          const int64_t mid = (lo + hi + 1) >> 1;
          if (moff[mid] - base <= e) lo = mid; else hi = mid - 1;
        }
        const int32_t j = rir[lo];
        const int64_t q = acp[j] + (e - (moff[lo] - base));
        const int32_t i = air[q];
        key[e] = ((uint64_t)(uint32_t)agg[i] << 32) | (uint32_t)e;
        val[e] = rv[i] * (aval ? aval[q] : 1.0) * rv[j];
      } else {
        key[e] = ~0ull;
      }
    }
    __syncthreads();
    for (int k = 2; k <= N; k <<= 1)
      for (int jj = k >> 1; jj > 0; jj >>= 1) {
        for (int tt = lane; tt < N / 2; tt += 64) {
          const int a = (tt / jj) * 2 * jj + (tt % jj), b = a + jj;
          const uint64_t x = key[a], y = key[b];
          if ((x > y) == ((a & k) == 0)) { key[a] = y; key[b] = x; }
        }
        __syncthreads();
      }
    int64_t run = 0;   // unique rows so far; written from `base` (this aggregate's entry range bounds them)
    for (int e0 = 0; e0 < t; e0 += 64) {
      const int e = e0 + lane;
      const bool head = e < t && (e == 0 || (key[e] >> 32) != (key[e - 1] >> 32));
      const uint64_t mask = __ballot(head);
      if (head) {
        const int64_t o = base + run + __popcll(mask & ((1ull << lane) - 1));
        const uint64_t r = key[e] >> 32;
        double v = val[key[e] & 0xffffffffu];
        for (int f = e + 1; f < t && (key[f] >> 32) == r; ++f) v += val[key[f] & 0xffffffffu];
        trow[o] = (int32_t)r;
        tval[o] = v;
      }
      run += __popcll(mask);
    }
    if (lane == 0) cnt[J] = run;
    __syncthreads();
  }
}

// C column J = the first cnt[J] entries of aggregate J's range in the scratch (16 lanes per column)
__global__ void k_rap_compact(int64_t nagg, const int64_t* __restrict__ rcp, const int64_t* __restrict__ moff,
                              const int64_t* __restrict__ ccp, const int32_t* __restrict__ trow,
                              const double* __restrict__ tval, int32_t* __restrict__ crow, double* __restrict__ cval) {
  const int sub = threadIdx.x & 15;
  for (int64_t J = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 4; J < nagg;
       J += ((int64_t)gridDim.x * blockDim.x) >> 4) {
    const int64_t src = moff[rcp[J]], dst = ccp[J], n = ccp[J + 1] - dst;
    for (int64_t x = sub; x < n; x += 16) {
      crow[dst + x] = trow[src + x];
      cval[dst + x] = tval[src + x];
    }
  }
}

// ---------------------------------------------------------------- the reference's RestrictionOp
// MTRand (psort-1.0/include/psort/MersenneTwister.h:137-147, 179-196, 283-314) = MT19937 with init_genrand
// seeding.  The state (624 words + read index) lives in HBM between launches; one workgroup draws the next
// *count values of the stream: each reload is the three data-parallel spans of the twist ([0,227) reads old
// words, [227,454) and [454,624) read words the previous span rewrote) staged in LDS.
constexpr int kMtN = 624;

__global__ void k_mt_seed(uint32_t seed, uint32_t* __restrict__ st) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    uint32_t x = seed;
    st[0] = x;
    for (uint32_t i = 1; i < kMtN; ++i) {
      x = 1812433253u * (x ^ (x >> 30)) + i;
      st[i] = x;
    }
    st[kMtN] = kMtN;   // read index: the first draw reloads
  }
}

__device__ __forceinline__ uint32_t mt_twist(uint32_t m, uint32_t s0, uint32_t s1) {
  return m ^ (((s0 & 0x80000000u) | (s1 & 0x7fffffffu)) >> 1) ^ ((s1 & 1u) ? 0x9908b0dfu : 0u);
}
__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  return y ^ (y >> 18);
}

// Two LDS copies of the state: a reload writes the new words into the other copy, so a span never
// overwrites words it still reads -- three barriers per 624 draws (one per dependent span); tempering reads
// the new copy while the next reload writes the old one.
__global__ void __launch_bounds__(256) k_mt_draw(uint32_t* __restrict__ st, const int64_t* __restrict__ count,
                                                 uint32_t* __restrict__ out) {
  __shared__ uint32_t buf[2][kMtN];
  const int t = threadIdx.x;
  int cur = 0;
  for (int i = t; i < kMtN; i += 256) buf[0][i] = st[i];
  uint32_t idx = st[kMtN];
  const int64_t n = *count;
  __syncthreads();
  for (int64_t done = 0; done < n;) {
    if (idx == kMtN) {
      const uint32_t* X = buf[cur];
      uint32_t* Y = buf[cur ^ 1];
      if (t < 227) Y[t] = mt_twist(X[t + 397], X[t], X[t + 1]);
      __syncthreads();
      if (t < 227) Y[t + 227] = mt_twist(Y[t], X[t + 227], X[t + 228]);
      __syncthreads();
      if (t < 169) Y[t + 454] = mt_twist(Y[t + 227], X[t + 454], X[t + 455]);
      else if (t == 169) Y[623] = mt_twist(Y[396], X[623], Y[0]);
      __syncthreads();
      cur ^= 1;
      idx = 0;
    }
    const uint32_t* Y = buf[cur];
    const int64_t take = min<int64_t>(kMtN - idx, n - done);
    for (int64_t k = t; k < take; k += 256) out[done + k] = mt_temper(Y[idx + k]);
    idx += (uint32_t)take;
    done += take;
  }
  __syncthreads();
  for (int i = t; i < kMtN; i += 256) st[i] = buf[cur][i];
  if (t == 0) st[kMtN] = idx;
}

// B = pattern(A) + pattern(A)^T without the diagonal (RestrictionOp.h:201-208): raw column counts ...
__global__ void k_sym_count(int64_t n, const int64_t* __restrict__ cp, const int32_t* __restrict__ ir,
                            unsigned long long* __restrict__ cnt) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
    unsigned long long own = 0;
    for (int64_t p = cp[j]; p < cp[j + 1]; ++p) {
      const int32_t i = ir[p];
      if (i == j) continue;
      ++own;
      atomicAdd(&cnt[i], 1ull);
    }
    if (own) atomicAdd(&cnt[j], own);
  }
}
// ... and the raw entries (column j gets row i, column i gets row j); rows are sorted and deduplicated after
__global__ void k_sym_fill(int64_t n, const int64_t* __restrict__ cp, const int32_t* __restrict__ ir,
                           unsigned long long* __restrict__ cursor, int32_t* __restrict__ rows) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x)
    for (int64_t p = cp[j]; p < cp[j + 1]; ++p) {
      const int32_t i = ir[p];
      if (i == j) continue;
      rows[atomicAdd(&cursor[j], 1ull)] = i;
      rows[atomicAdd(&cursor[i], 1ull)] = (int32_t)j;
    }
}

constexpr uint64_t kNoVal = ~0ull;

// flag[v] = cand[v] (int64, for the candidate ranks)
__global__ void k_flag64(int64_t n, const uint8_t* __restrict__ f, int64_t* __restrict__ out) {
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x)
    out[v] = f[v];
}
// r[v] = this round's draw of candidate v (the pos[v]-th value of the round), else none
__global__ void k_cand_vals(int64_t n, const uint8_t* __restrict__ cand, const int64_t* __restrict__ pos,
                            const uint32_t* __restrict__ draw, uint64_t* __restrict__ r) {
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x)
    r[v] = cand[v] ? (uint64_t)draw[pos[v]] : kNoVal;
}
// out[v] = min over neighbours u of in[u] (SpMV with Select2ndMinSR, RestrictionOp.h:146-147)
__global__ void k_nbr_min(int64_t n, const int64_t* __restrict__ cp, const int32_t* __restrict__ ir,
                          const uint64_t* __restrict__ in, uint64_t* __restrict__ out) {
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
    uint64_t m = kNoVal;
    for (int64_t p = cp[v]; p < cp[v + 1]; ++p) m = min(m, in[ir[p]]);
    out[v] = m;
  }
}
// new members: candidates whose draw is <= the 1- and 2-hop minimum (RestrictionOp.h:149-161)
__global__ void k_mis_new(int64_t n, const uint8_t* __restrict__ cand, const uint64_t* __restrict__ r,
                          const uint64_t* __restrict__ m1, const uint64_t* __restrict__ m2, uint8_t* __restrict__ fresh) {
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x)
    fresh[v] = cand[v] && r[v] <= min(m1[v], m2[v]);
}
// out[v] = 1 iff a neighbour u has in[u] (SpMV of the new members and of their neighbours, :170-171)
__global__ void k_nbr_any(int64_t n, const int64_t* __restrict__ cp, const int32_t* __restrict__ ir,
                          const uint8_t* __restrict__ in, uint8_t* __restrict__ out) {
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
    uint8_t f = 0;
    for (int64_t p = cp[v]; p < cp[v + 1] && !f; ++p) f = in[ir[p]];
    out[v] = f;
  }
}
// members leave the candidates with their 1- and 2-hop neighbours and join the set (:164-189)
__global__ void k_mis_round(int64_t n, const uint8_t* __restrict__ fresh, const uint8_t* __restrict__ nb1,
                            const uint8_t* __restrict__ nb2, uint8_t* __restrict__ cand, uint8_t* __restrict__ mis,
                            int64_t* __restrict__ left) {
  int64_t c = 0;
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t f = fresh[v];
    const uint8_t k = cand[v] && !f && !nb1[v] && !nb2[v];
    cand[v] = k;
    if (f) mis[v] = 1;
    c += k;
  }
  c = wave_sum64(c);
  if (lane_id() == 0 && c) atomicAdd((unsigned long long*)left, (unsigned long long)c);
}
// parent[v] = v for set members, else the (unique) set member among the neighbours (MIS2verifySR and the union
// with mis2, :216-222), else -1; flag = has a parent
__global__ void k_mis_parent(int64_t n, const int64_t* __restrict__ cp, const int32_t* __restrict__ ir,
                             const uint8_t* __restrict__ mis, int64_t* __restrict__ parent, int64_t* __restrict__ has,
                             int64_t* __restrict__ misflag) {
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
    int64_t p = -1;
    if (mis[v]) {
      p = v;
    } else {
      for (int64_t q = cp[v]; q < cp[v + 1]; ++q)
        if (mis[ir[q]]) { p = p < 0 ? ir[q] : min<int64_t>(p, ir[q]); }
    }
    parent[v] = p;
    has[v] = p >= 0;
    misflag[v] = mis[v];
  }
}
// key[v] = (draw, larger vertex first) of parented vertices (mis2neigh_p, :225-229)
__global__ void k_parent_keys(int64_t n, const int64_t* __restrict__ has, const int64_t* __restrict__ pos,
                              const uint32_t* __restrict__ draw, uint64_t* __restrict__ key) {
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x)
    key[v] = has[v] ? ((uint64_t)draw[pos[v]] << 32 | (uint64_t)(0xffffffffu - (uint32_t)v)) : kNoVal;
}
// aggregate column of v: its parent, else the parent of the neighbour with the smallest draw (Select2ndRandSR,
// :63-84, 233-247); the column is the parent's rank among the set members, permuted (RandPerm, :268-275)
__global__ void k_restrict_cols(int64_t n, const int64_t* __restrict__ parent, const uint64_t* __restrict__ best,
                                const int64_t* __restrict__ misrank, const int32_t* __restrict__ inv,
                                int32_t* __restrict__ agg, unsigned long long* __restrict__ colcnt,
                                int64_t* __restrict__ bad) {
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
    int64_t p = parent[v];
    if (p < 0 && best[v] != kNoVal) p = parent[0xffffffffu - (uint32_t)(best[v] & 0xffffffffu)];
    if (p < 0) {
      agg[v] = -1;
      atomicAdd((unsigned long long*)bad, 1ull);
      continue;
    }
    const int32_t a = inv[misrank[p]];
    agg[v] = a;
    atomicAdd(&colcnt[a], 1ull);
  }
}

template <class Buf>   // DevBuf (persistent workspace) or PoolBuf
cbg_status scan_counts_async(hipStream_t st, int64_t n, const int64_t* cnt, int64_t* out, int64_t* total_dev,
                             Buf* tiles) {
  const int64_t ntiles = (n + kScanTile - 1) / kScanTile;
  HIPCHK(tiles->reserve(sizeof(int64_t) * (ntiles + 1)));
  if (n > 0) {
    k_scan_tiles<<<(int)ntiles, 256, 0, st>>>(n, cnt, (int64_t*)tiles->p);
    k_scan_sums<<<1, 1024, 0, st>>>(ntiles, (int64_t*)tiles->p, total_dev);
    k_scan_apply<<<(int)ntiles, 256, 0, st>>>(n, cnt, (int64_t*)tiles->p, out);
  } else {
    HIPCHK(hipMemsetAsync(out, 0, sizeof(int64_t), st));
    HIPCHK(hipMemsetAsync(total_dev, 0, sizeof(int64_t), st));
  }
  HIPCHK(hipGetLastError());
  return CBG_OK;
}

}  // namespace

extern "C" cbg_status cbg_mis2_restriction(cbg_ctx* ctx, const cbg_dcsc_view* Gv, uint64_t seed, cbg_csc_result* R,
                                           cbg_csc_result* RT, int64_t* nagg_out) {
  if (!ctx || !Gv || !R) return CBG_EINVAL;
  if (Gv->nrow != Gv->ncol) return CBG_EDIM;
  HIPCHK(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  DevBuf sb[5];
  DevCsc<double> G;
  CBGCHK(stage<double>(ctx, Gv, sb, &G));
  const int64_t n = G.ncol;
  if (n >= INT32_MAX) return CBG_EUNSUP;
  // scratch from the context's caching pool (stream-ordered reuse; no hipMalloc/hipFree per call)
  PoolBuf key, m1, m2, st8, fr, c1, c2, sc, tiles;
  for (PoolBuf* b : {&key, &m1, &m2, &st8, &fr, &c1, &c2, &sc, &tiles}) b->pool = ctx->pool;
  HIPCHK(key.reserve(8 * (n + 1)));
  HIPCHK(m1.reserve(8 * (n + 1)));
  HIPCHK(m2.reserve(8 * (n + 1)));
  HIPCHK(st8.reserve(n + 1));
  HIPCHK(fr.reserve(n + 1));
  HIPCHK(c1.reserve(n + 1));
  HIPCHK(c2.reserve(n + 1));
  HIPCHK(sc.reserve(64));
  const int g = (int)grid_for(n, 256, kMaxGrid * 4);
  int8_t* state = st8.as<int8_t>();
  unsigned long long* und = sc.as<unsigned long long>();
  k_mis_keys<<<g, 256, 0, st>>>(n, seed, key.as<uint64_t>(), state);
  for (int round = 0; n > 0; ++round) {
    if (round > 4096) return CBG_EDEVICE;   // every round roots the largest undecided key: cannot happen
    k_nbr_max<true><<<g, 256, 0, st>>>(n, G.cp, G.ir, key.as<uint64_t>(), state, 0, m1.as<uint64_t>());
    k_nbr_max<false><<<g, 256, 0, st>>>(n, G.cp, G.ir, m1.as<uint64_t>(), state, 0, m2.as<uint64_t>());
    k_mis_select<<<g, 256, 0, st>>>(n, key.as<uint64_t>(), m2.as<uint64_t>(), state, fr.as<uint8_t>());
    k_nbr_or<<<g, 256, 0, st>>>(n, G.cp, G.ir, fr.as<uint8_t>(), c1.as<uint8_t>());
    k_nbr_or<<<g, 256, 0, st>>>(n, G.cp, G.ir, c1.as<uint8_t>(), c2.as<uint8_t>());
    HIPCHK(hipMemsetAsync(und, 0, 8, st));
    k_mis_update<<<g, 256, 0, st>>>(n, fr.as<uint8_t>(), c2.as<uint8_t>(), state, und);
    HIPCHK(hipGetLastError());
    unsigned long long left = 0;
    HIPCHK(hipMemcpyAsync(&left, und, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (left == 0) break;
  }
  // aggregates: nearest root within distance 1, else 2 (m1/m2 reused for the root-key maxima)
  PoolBuf rk, isr, rid, agg, cnt;
  for (PoolBuf* b : {&rk, &isr, &rid, &agg, &cnt}) b->pool = ctx->pool;
  HIPCHK(rk.reserve(8 * (n + 1)));
  HIPCHK(isr.reserve(8 * (n + 1)));
  HIPCHK(rid.reserve(8 * (n + 1)));
  HIPCHK(agg.reserve(4 * (n + 1)));
  k_root_keys<<<g, 256, 0, st>>>(n, key.as<uint64_t>(), state, rk.as<uint64_t>(), isr.as<int64_t>());
  k_nbr_max<false><<<g, 256, 0, st>>>(n, G.cp, G.ir, rk.as<uint64_t>(), state, 0, m1.as<uint64_t>());
  k_nbr_max<false><<<g, 256, 0, st>>>(n, G.cp, G.ir, m1.as<uint64_t>(), state, 0, m2.as<uint64_t>());
  HIPCHK(hipGetLastError());
  CBGCHK(scan_counts_async(st, n, isr.as<int64_t>(), rid.as<int64_t>(), (int64_t*)(sc.as<char>() + 8), &tiles));
  int64_t nagg = 0;
  HIPCHK(hipMemcpyAsync(&nagg, sc.as<char>() + 8, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  HIPCHK(cnt.reserve(8 * (2 * nagg + 2)));
  unsigned long long* colcnt = cnt.as<unsigned long long>();
  unsigned long long* cursor = colcnt + nagg + 1;
  HIPCHK(hipMemsetAsync(cnt.p, 0, 8 * (2 * nagg + 2), st));
  k_assign<<<g, 256, 0, st>>>(n, m1.as<uint64_t>(), m2.as<uint64_t>(), rid.as<int64_t>(), agg.as<int32_t>(), colcnt);
  HIPCHK(hipGetLastError());
  // R (n x nagg): members of each aggregate, row-sorted by the duplicate-summing product (values 1)
  PoolBuf rawcp, rows;
  rawcp.pool = rows.pool = ctx->pool;
  HIPCHK(rawcp.reserve(8 * (nagg + 1)));
  HIPCHK(rows.reserve(4 * (n + 1)));
  CBGCHK(scan_counts_async(st, nagg, (const int64_t*)colcnt, rawcp.as<int64_t>(), (int64_t*)(sc.as<char>() + 16),
                           &tiles));
  if (nagg) HIPCHK(hipMemcpyAsync(cursor, rawcp.p, 8 * nagg, hipMemcpyDeviceToDevice, st));
  k_scatter_members<<<g, 256, 0, st>>>(n, agg.as<int32_t>(), cursor, rows.as<int32_t>());
  HIPCHK(hipGetLastError());
  CBGCHK(dedup_columns(ctx, n, nagg, n, rawcp.as<int64_t>(), rows.as<int32_t>(), nullptr, R));
  R->multiplies = 0;
  if (RT) {   // R^T (nagg x n): column v holds the single row agg(v)
    std::unique_ptr<Owner> own(new Owner(ctx->pool));
    HIPCHK(own->cp.reserve(8 * (n + 1)));
    HIPCHK(own->ir.reserve(4 * (n + 1)));
    HIPCHK(own->val.reserve(8 * (n + 1)));
    k_rt<<<(int)grid_for(n + 1, 256, kMaxGrid * 4), 256, 0, st>>>(n, agg.as<int32_t>(), own->cp.as<int64_t>(),
                                                                  own->ir.as<int32_t>(), own->val.as<double>());
    HIPCHK(hipGetLastError());
    memset(RT, 0, sizeof(*RT));
    RT->nrow = nagg; RT->ncol = n; RT->nnz = n;
    RT->colptr = own->cp.as<int64_t>(); RT->row = own->ir.as<int32_t>(); RT->val = own->val.p;
    RT->val_type = CBG_F64;
    RT->_owner = own.release();
  }
  HIPCHK(hipStreamSynchronize(st));
  if (nagg_out) *nagg_out = nagg;
  return CBG_OK;
}

// The reference's RestrictionOp (3DSpGEMM/RestrictionOp.h:196-291) at one rank: MIS2 (:116-193) with the
// MTRand stream seeded by mt_seed, parents, Select2ndRandSR aggregation and RandPerm of the aggregate columns
// (FullyDistVec.cpp:783-900: std::shuffle of 0..nagg-1 with std::default_random_engine(perm_seed), the one
// host step -- the reference's RandPerm is host code too, O(nagg)).  The reference's DETERMINISTIC seeds are
// mt_seed = 1, perm_seed = 1383098845.  Every vertex-parallel step is one thread per vertex over B's CSC;
// the draws of a round are ranked by a scan of the candidate flags, so the round needs no host copy except
// the count of remaining candidates.
extern "C" cbg_status cbg_restriction_op(cbg_ctx* ctx, const cbg_dcsc_view* Av, uint32_t mt_seed, uint32_t perm_seed,
                                         cbg_csc_result* R, cbg_csc_result* RT, int64_t* nagg_out) {
  if (!ctx || !Av || !R) return CBG_EINVAL;
  if (Av->nrow != Av->ncol) return CBG_EDIM;
  HIPCHK(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  DevBuf sb[5];
  DevCsc<double> A;
  CBGCHK(stage<double>(ctx, Av, sb, &A));
  const int64_t n = A.ncol;
  if (n >= INT32_MAX) return CBG_EUNSUP;
  const int g = (int)grid_for(std::max<int64_t>(n, 1), 256, kMaxGrid * 4);
  PoolBuf cnt, tiles, rows, sc, mt;
  for (PoolBuf* b : {&cnt, &tiles, &rows, &sc, &mt}) b->pool = ctx->pool;
  HIPCHK(sc.reserve(64));
  int64_t* scal = sc.as<int64_t>();   // [0] raw B entries [1] draws this round [2] left [3] parented [4] nagg [5] bad
  HIPCHK(hipMemsetAsync(scal, 0, 64, st));
  // B: symmetric, loop-free pattern of A, rows sorted and unique per column
  HIPCHK(cnt.reserve(8 * (2 * n + 2)));
  unsigned long long* bcnt = cnt.as<unsigned long long>();
  unsigned long long* cursor = bcnt + n + 1;
  HIPCHK(hipMemsetAsync(bcnt, 0, 8 * (n + 1), st));
  PoolBuf rawcp;
  rawcp.pool = ctx->pool;
  HIPCHK(rawcp.reserve(8 * (n + 1)));
  if (n) k_sym_count<<<g, 256, 0, st>>>(n, A.cp, A.ir, bcnt);
  HIPCHK(hipGetLastError());
  CBGCHK(scan_counts_async(st, n, (const int64_t*)bcnt, rawcp.as<int64_t>(), scal, &tiles));
  int64_t nraw = 0;
  HIPCHK(hipMemcpyAsync(&nraw, scal, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  HIPCHK(rows.reserve(4 * (nraw + 1)));
  if (n) HIPCHK(hipMemcpyAsync(cursor, rawcp.p, 8 * n, hipMemcpyDeviceToDevice, st));
  if (n) k_sym_fill<<<g, 256, 0, st>>>(n, A.cp, A.ir, cursor, rows.as<int32_t>());
  HIPCHK(hipGetLastError());
  cbg_csc_result Bres;
  CBGCHK(dedup_columns(ctx, n, n, nraw, rawcp.as<int64_t>(), rows.as<int32_t>(), nullptr, &Bres));
  std::unique_ptr<Owner> bown((Owner*)Bres._owner);
  const int64_t* bcp = Bres.colptr;
  const int32_t* bir = Bres.row;
  // MIS2
  PoolBuf cand, mis, fresh, nb1, nb2, flag, pos, draw, r, m1, m2;
  for (PoolBuf* b : {&cand, &mis, &fresh, &nb1, &nb2, &flag, &pos, &draw, &r, &m1, &m2}) b->pool = ctx->pool;
  for (PoolBuf* b : {&cand, &mis, &fresh, &nb1, &nb2}) HIPCHK(b->reserve(n + 1));
  for (PoolBuf* b : {&flag, &pos, &r, &m1, &m2}) HIPCHK(b->reserve(8 * (n + 1)));
  HIPCHK(draw.reserve(4 * (n + 1)));
  HIPCHK(mt.reserve(4 * (kMtN + 1)));
  HIPCHK(hipMemsetAsync(cand.p, 1, n + 1, st));
  HIPCHK(hipMemsetAsync(mis.p, 0, n + 1, st));
  k_mt_seed<<<1, 64, 0, st>>>(mt_seed, mt.as<uint32_t>());
  HIPCHK(hipGetLastError());
  int64_t left = n;
  for (int round = 0; left > 0; ++round) {
    if (round > 4096) return CBG_EDEVICE;   // every round admits the smallest draw: cannot happen
    k_flag64<<<g, 256, 0, st>>>(n, cand.as<uint8_t>(), flag.as<int64_t>());
    CBGCHK(scan_counts_async(st, n, flag.as<int64_t>(), pos.as<int64_t>(), scal + 1, &tiles));
    k_mt_draw<<<1, 256, 0, st>>>(mt.as<uint32_t>(), scal + 1, draw.as<uint32_t>());
    k_cand_vals<<<g, 256, 0, st>>>(n, cand.as<uint8_t>(), pos.as<int64_t>(), draw.as<uint32_t>(), r.as<uint64_t>());
    k_nbr_min<<<g, 256, 0, st>>>(n, bcp, bir, r.as<uint64_t>(), m1.as<uint64_t>());
    k_nbr_min<<<g, 256, 0, st>>>(n, bcp, bir, m1.as<uint64_t>(), m2.as<uint64_t>());
    k_mis_new<<<g, 256, 0, st>>>(n, cand.as<uint8_t>(), r.as<uint64_t>(), m1.as<uint64_t>(), m2.as<uint64_t>(),
                                 fresh.as<uint8_t>());
    k_nbr_any<<<g, 256, 0, st>>>(n, bcp, bir, fresh.as<uint8_t>(), nb1.as<uint8_t>());
    k_nbr_any<<<g, 256, 0, st>>>(n, bcp, bir, nb1.as<uint8_t>(), nb2.as<uint8_t>());
    HIPCHK(hipMemsetAsync(scal + 2, 0, 8, st));
    k_mis_round<<<g, 256, 0, st>>>(n, fresh.as<uint8_t>(), nb1.as<uint8_t>(), nb2.as<uint8_t>(), cand.as<uint8_t>(),
                                   mis.as<uint8_t>(), scal + 2);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(&left, scal + 2, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  }
  // parents, their draws, the aggregation of the unparented vertices, the MIS ranks (m1 = parent,
  // flag = has-parent, r = MIS flags as int64 -> pos/misrank)
  PoolBuf misrank;
  misrank.pool = ctx->pool;
  HIPCHK(misrank.reserve(8 * (n + 1)));
  k_mis_parent<<<g, 256, 0, st>>>(n, bcp, bir, mis.as<uint8_t>(), m1.as<int64_t>(), flag.as<int64_t>(),
                                  r.as<int64_t>());
  HIPCHK(hipGetLastError());
  CBGCHK(scan_counts_async(st, n, flag.as<int64_t>(), pos.as<int64_t>(), scal + 3, &tiles));
  CBGCHK(scan_counts_async(st, n, r.as<int64_t>(), misrank.as<int64_t>(), scal + 4, &tiles));
  k_mt_draw<<<1, 256, 0, st>>>(mt.as<uint32_t>(), scal + 3, draw.as<uint32_t>());
  k_parent_keys<<<g, 256, 0, st>>>(n, flag.as<int64_t>(), pos.as<int64_t>(), draw.as<uint32_t>(), m2.as<uint64_t>());
  k_nbr_min<<<g, 256, 0, st>>>(n, bcp, bir, m2.as<uint64_t>(), r.as<uint64_t>());
  HIPCHK(hipGetLastError());
  int64_t nagg = 0;
  HIPCHK(hipMemcpyAsync(&nagg, scal + 4, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  // RandPerm of the aggregate columns: new column j is old column perm[j]; inv[perm[j]] = j
  std::vector<int64_t> perm((size_t)nagg);
  std::iota(perm.begin(), perm.end(), 0);
  std::default_random_engine gen(perm_seed);
  std::shuffle(perm.begin(), perm.end(), gen);
  std::vector<int32_t> inv((size_t)nagg + 1);
  for (int64_t j = 0; j < nagg; ++j) inv[(size_t)perm[(size_t)j]] = (int32_t)j;
  PoolBuf dinv, agg, ccnt, rcp, members;
  for (PoolBuf* b : {&dinv, &agg, &ccnt, &rcp, &members}) b->pool = ctx->pool;
  HIPCHK(dinv.reserve(4 * (nagg + 1)));
  HIPCHK(agg.reserve(4 * (n + 1)));
  HIPCHK(ccnt.reserve(8 * (2 * nagg + 2)));
  HIPCHK(rcp.reserve(8 * (nagg + 1)));
  HIPCHK(members.reserve(4 * (n + 1)));
  HIPCHK(hipMemcpyAsync(dinv.p, inv.data(), 4 * (nagg + 1), hipMemcpyHostToDevice, st));
  unsigned long long* colcnt = ccnt.as<unsigned long long>();
  unsigned long long* ccur = colcnt + nagg + 1;
  HIPCHK(hipMemsetAsync(colcnt, 0, 8 * (nagg + 1), st));
  k_restrict_cols<<<g, 256, 0, st>>>(n, m1.as<int64_t>(), r.as<uint64_t>(), misrank.as<int64_t>(), dinv.as<int32_t>(),
                                     agg.as<int32_t>(), colcnt, scal + 5);
  HIPCHK(hipGetLastError());
  CBGCHK(scan_counts_async(st, nagg, (const int64_t*)colcnt, rcp.as<int64_t>(), scal + 6, &tiles));
  if (nagg) HIPCHK(hipMemcpyAsync(ccur, rcp.p, 8 * nagg, hipMemcpyDeviceToDevice, st));
  k_scatter_members<<<g, 256, 0, st>>>(n, agg.as<int32_t>(), ccur, members.as<int32_t>());
  HIPCHK(hipGetLastError());
  int64_t bad = 0;
  HIPCHK(hipMemcpyAsync(&bad, scal + 5, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));   // inv (host) is read; bad is known
  if (bad) return CBG_EDEVICE;        // a vertex beyond distance 2 of the set: not a maximal MIS-2
  CBGCHK(dedup_columns(ctx, n, nagg, n, rcp.as<int64_t>(), members.as<int32_t>(), nullptr, R));
  R->multiplies = 0;
  if (RT) {   // R^T (nagg x n): column v holds the single row agg(v)
    std::unique_ptr<Owner> own(new Owner(ctx->pool));
    HIPCHK(own->cp.reserve(8 * (n + 1)));
    HIPCHK(own->ir.reserve(4 * (n + 1)));
    HIPCHK(own->val.reserve(8 * (n + 1)));
    k_rt<<<(int)grid_for(n + 1, 256, kMaxGrid * 4), 256, 0, st>>>(n, agg.as<int32_t>(), own->cp.as<int64_t>(),
                                                                  own->ir.as<int32_t>(), own->val.as<double>());
    HIPCHK(hipGetLastError());
    memset(RT, 0, sizeof(*RT));
    RT->nrow = nagg; RT->ncol = n; RT->nnz = n;
    RT->colptr = own->cp.as<int64_t>(); RT->row = own->ir.as<int32_t>(); RT->val = own->val.p;
    RT->val_type = CBG_F64;
    RT->_owner = own.release();
  }
  HIPCHK(hipStreamSynchronize(st));
  if (nagg_out) *nagg_out = nagg;
  return CBG_OK;
}

// C = A^T (SpDCCols::Transpose, SpDCCols.cpp:845): per-row counts, scatter of (column, value) into the rows'
// columns, then the duplicate-free row sort of dedup_columns.  PlusTimes<double> values (or a pattern).
__global__ void k_row_counts(int64_t nnz, const int32_t* __restrict__ ir, unsigned long long* __restrict__ cnt) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < nnz; p += (int64_t)gridDim.x * blockDim.x)
    atomicAdd(&cnt[ir[p]], 1ull);
}
__global__ void k_transpose_fill(int64_t ncol, const int64_t* __restrict__ cp, const int32_t* __restrict__ ir,
                                 const double* __restrict__ val, unsigned long long* __restrict__ cursor,
                                 int32_t* __restrict__ orow, double* __restrict__ oval) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < ncol; j += (int64_t)gridDim.x * blockDim.x)
    for (int64_t p = cp[j]; p < cp[j + 1]; ++p) {
      const unsigned long long o = atomicAdd(&cursor[ir[p]], 1ull);
      orow[o] = (int32_t)j;
      if (oval) oval[o] = val ? val[p] : 1.0;
    }
}

extern "C" cbg_status cbg_transpose(cbg_ctx* ctx, const cbg_dcsc_view* Av, cbg_csc_result* C) {
  if (!ctx || !Av || !C) return CBG_EINVAL;
  if (Av->val && Av->val_type != CBG_F64) return CBG_EUNSUP;
  HIPCHK(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  DevBuf sb[5];
  DevCsc<double> A;
  CBGCHK(stage<double>(ctx, Av, sb, &A));
  const int64_t m = A.nrow, n = A.ncol, nnz = A.nnz;
  if (n >= INT32_MAX) return CBG_EUNSUP;
  PoolBuf cnt, ocp, rows, vals, tiles, sc;
  for (PoolBuf* b : {&cnt, &ocp, &rows, &vals, &tiles, &sc}) b->pool = ctx->pool;
  HIPCHK(cnt.reserve(8 * (2 * m + 2)));
  HIPCHK(ocp.reserve(8 * (m + 1)));
  HIPCHK(rows.reserve(4 * (nnz + 1)));
  HIPCHK(vals.reserve(8 * (nnz + 1)));
  HIPCHK(sc.reserve(16));
  unsigned long long* c = cnt.as<unsigned long long>();
  unsigned long long* cur = c + m + 1;
  HIPCHK(hipMemsetAsync(c, 0, 8 * (m + 1), st));
  if (nnz) k_row_counts<<<(int)grid_for(nnz, 256, kMaxGrid * 4), 256, 0, st>>>(nnz, A.ir, c);
  HIPCHK(hipGetLastError());
  CBGCHK(scan_counts_async(st, m, (const int64_t*)c, ocp.as<int64_t>(), sc.as<int64_t>(), &tiles));
  if (m) HIPCHK(hipMemcpyAsync(cur, ocp.p, 8 * m, hipMemcpyDeviceToDevice, st));
  const bool has_val = A.val != nullptr;
  if (n) k_transpose_fill<<<(int)grid_for(n, 256, kMaxGrid * 4), 256, 0, st>>>(n, A.cp, A.ir, A.val, cur,
                                                                               rows.as<int32_t>(), vals.as<double>());
  HIPCHK(hipGetLastError());
  CBGCHK(dedup_columns(ctx, n, m, nnz, ocp.as<int64_t>(), rows.as<int32_t>(), has_val ? vals.as<double>() : nullptr, C));
  C->multiplies = 0;
  return CBG_OK;
}

extern "C" cbg_status cbg_galerkin_rap(cbg_ctx* ctx, const cbg_dcsc_view* Av, const cbg_dcsc_view* Rv,
                                       cbg_csc_result* C) {
  if (!ctx || !Av || !Rv || !C) return CBG_EINVAL;
  if (Av->nrow != Av->ncol || Rv->nrow != Av->ncol) return CBG_EDIM;   // R^T A R: A square, R n x nagg
  HIPCHK(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  DevBuf sa[5], sr[5];
  DevCsc<double> A, R;
  CBGCHK(stage<double>(ctx, Av, sa, &A));
  CBGCHK(stage<double>(ctx, Rv, sr, &R));
  const int64_t n = A.ncol, nagg = R.ncol, nnzr = R.nnz;
  // For an aggregation every column of A is one member, so the entries to reduce are exactly nnz(A):
  // the scratch is sized up front and the aggregation check rides on the single read-back below.
  const int64_t nraw = A.nnz;
  DevBuf* w = ctx->gal;   // persistent workspace: no allocation on the hot path
  HIPCHK(w[0].reserve(4 * (n + 1)));            // agg
  HIPCHK(w[1].reserve(8 * (n + 1)));            // rv
  HIPCHK(w[2].reserve(4 * (n + 1)));            // seen
  HIPCHK(w[3].reserve(8 * (std::max(nnzr, nagg) + 1)));   // member lengths, then per-aggregate counts
  HIPCHK(w[4].reserve(8 * (nnzr + 1)));         // member offsets
  HIPCHK(w[5].reserve(12 * (nraw + 1)));        // scratch rows + values
  HIPCHK(w[6].reserve(64));                     // [0] bad rows [1] raw total [2] overflow [3] nnz(C)
  int32_t* agg = w[0].as<int32_t>();
  double* rv = w[1].as<double>();
  int64_t* len = w[3].as<int64_t>();
  int64_t* moff = w[4].as<int64_t>();
  double* tval = w[5].as<double>();
  int32_t* trow = (int32_t*)(tval + nraw + 1);
  int64_t* sc = w[6].as<int64_t>();
  HIPCHK(hipMemsetAsync(w[2].p, 0, 4 * (n + 1), st));
  HIPCHK(hipMemsetAsync(sc, 0, 64, st));
  const int g = (int)grid_for(std::max(std::max(n, nagg), nnzr), 256, kMaxGrid * 4);
  k_r_rows<<<g, 256, 0, st>>>(nagg, R.cp, R.ir, R.val, agg, rv, w[2].as<unsigned int>());
  k_count_bad<<<g, 256, 0, st>>>(n, w[2].as<unsigned int>(), (unsigned long long*)sc);
  k_member_len<<<g, 256, 0, st>>>(nnzr, R.ir, A.cp, len);
  HIPCHK(hipGetLastError());
  CBGCHK(scan_counts_async(st, nnzr, len, moff, sc + 1, &w[7]));
  const int ga = (int)std::min<int64_t>(std::max<int64_t>(nagg, 1), 65536);
  std::unique_ptr<Owner> own(new Owner(ctx->pool));
  HIPCHK(own->cp.reserve(8 * (nagg + 1)));
  if (nnzr == n) {
    // aggregates above kRapCap entries are listed for the kRapCapBig pass (device count, no read-back)
    HIPCHK(w[8].reserve(4 * (nagg + 1)));
    unsigned long long* nbig = (unsigned long long*)(sc + 4);
    k_rap_agg<kRapCap><<<ga, 64, 0, st>>>(nagg, nullptr, nullptr, w[8].as<int32_t>(), nbig, R.cp, R.ir, A.cp, A.ir,
                                          A.val, agg, rv, moff, len, trow, tval, nraw, (unsigned long long*)(sc + 2));
    k_rap_agg<kRapCapBig><<<1024, 64, 0, st>>>(nagg, w[8].as<int32_t>(), nbig, nullptr, nullptr, R.cp, R.ir, A.cp,
                                               A.ir, A.val, agg, rv, moff, len, trow, tval, nraw,
                                               (unsigned long long*)(sc + 2));
    HIPCHK(hipGetLastError());
    CBGCHK(scan_counts_async(st, nagg, len, own->cp.as<int64_t>(), sc + 3, &w[7]));
  }
  int64_t h[4] = {0, 0, 0, 0};
  HIPCHK(hipMemcpyAsync(h, sc, 32, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (nnzr != n || h[0] || h[1] != nraw) return CBG_EUNSUP;   // not an aggregation: two products instead
  if (h[2]) return CBG_EUNSUP;   // an aggregate gathers more than kRapCapBig entries: two products instead
  const int64_t nnzc = h[3];
  HIPCHK(own->ir.reserve(4 * (nnzc + 1)));
  HIPCHK(own->val.reserve(8 * (nnzc + 1)));
  k_rap_compact<<<(int)grid_for(nagg * 16, 256, kMaxGrid * 4), 256, 0, st>>>(
      nagg, R.cp, moff, own->cp.as<int64_t>(), trow, tval, own->ir.as<int32_t>(), own->val.as<double>());
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(st));
  memset(C, 0, sizeof(*C));
  C->nrow = nagg; C->ncol = nagg; C->nnz = nnzc;
  C->colptr = own->cp.as<int64_t>(); C->row = own->ir.as<int32_t>(); C->val = own->val.p;
  C->val_type = CBG_F64;
  C->multiplies = nraw;   // one scaled copy per nonzero of A (the fused pass)
  C->_owner = own.release();
  return CBG_OK;
}
