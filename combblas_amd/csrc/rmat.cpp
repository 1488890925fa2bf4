// rmat.cpp -- deterministic Graph500-style Kronecker (R-MAT) generator, host side.
//
// Semantics follow the reference's packed Graph500 path (include/CombBLAS/RefGen21.h:102-225 and
// DistEdgeList::GenGraph500Data, DistEdgeList.cpp:223-280) and the SpParMat(DistEdgeList) build
// (SpParMat.cpp:3082-3196, SpTuples.cpp:66-115):
//   * 16*2^scale edges, initiator a,b,c,d = 0.57,0.19,0.19,0.05 (RefGen21.h:73-75, numerators /10000)
//   * per level a quadrant draw; "clip-and-flip" keeps src <= tgt while both halves coincide
//     (RefGen21.h:206-214), so the unscrambled graph is upper triangular
//   * vertex ids scrambled by a bijection of [0, 2^scale)
//   * edge (src, tgt) -> A(src, tgt); duplicate edges summed, value = multiplicity (f64), loops kept.
// The random stream is our own counter-based hash (splitmix64 of (seed, edge, level)), so matrices are
// statistically equivalent to (not bit-identical with) the reference's MRG stream; golden parity
// tests use reference-generated inputs stored as fixtures instead.
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include <algorithm>
#include "cbgpu.h"

namespace {

inline uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// bijection on [0, 2^s): odd multiply, add, xor-shift, odd multiply (all invertible mod 2^s)
inline uint64_t scramble(uint64_t v, int s, uint64_t k0, uint64_t k1) {
  const uint64_t mask = (s >= 64) ? ~0ull : ((1ull << s) - 1);
  v = (v * (k0 | 1ull) + k1) & mask;
  v ^= v >> ((s + 1) / 2);
  v = (v * ((k1 << 1) | 1ull)) & mask;
  v ^= v >> ((s + 2) / 3);
  v = (v * 0x9E3779B97F4A7C15ull + k0) & mask;
  return v;
}

inline void make_edge(uint64_t seed, uint64_t e, int scale, uint64_t k0, uint64_t k1, uint32_t* src, uint32_t* tgt) {
  uint64_t bs = 0, bt = 0;
  uint64_t state = mix64(seed ^ mix64(e));
  for (int lvl = 0; lvl < scale; ++lvl) {
    if ((lvl & 1) == 0) state = mix64(state + (uint64_t)lvl);
    const uint32_t draw = (uint32_t)(state >> ((lvl & 1) ? 32 : 0));
    const uint32_t val = draw % 10000u;          // INITIATOR_DENOMINATOR
    int sq;                                      // generate_4way_bernoulli quadrant order
    if (val < 1900u) sq = 1;                     // b
    else if (val < 3800u) sq = 2;                // c
    else if (val < 9500u) sq = 0;                // a (5700)
    else sq = 3;                                 // d
    int so = sq / 2, to = sq % 2;
    if (bs == bt && so > to) { int t = so; so = to; to = t; }   // clip-and-flip
    const uint64_t half = 1ull << (scale - 1 - lvl);
    bs += half * so;
    bt += half * to;
  }
  *src = (uint32_t)scramble(bs, scale, k0, k1);
  *tgt = (uint32_t)scramble(bt, scale, k0, k1);
}

}  // namespace

extern "C" cbg_status cbg_rmat_host(int32_t scale, int32_t edgefactor, uint64_t seed, cbg_host_csc* out) {
  if (!out || scale < 1 || scale > 31 || edgefactor < 1) return CBG_EINVAL;
  memset(out, 0, sizeof(*out));
  const int64_t n = 1ll << scale;
  const int64_t m = (int64_t)edgefactor << scale;
  const uint64_t k0 = mix64(seed * 0x51ED2705ull + 1), k1 = mix64(seed + 0xA5A5A5A5ull);
  std::vector<uint32_t> src(m), tgt(m);
#pragma omp parallel for schedule(static)
  for (int64_t e = 0; e < m; ++e) make_edge(seed, (uint64_t)e, scale, k0, k1, &src[e], &tgt[e]);
  // counting sort by column (tgt), then per-column row sort + duplicate merge
  std::vector<int64_t> cnt(n + 1, 0);
  for (int64_t e = 0; e < m; ++e) cnt[tgt[e] + 1]++;
  for (int64_t c = 0; c < n; ++c) cnt[c + 1] += cnt[c];
  std::vector<uint32_t> rows(m);
  {
    std::vector<int64_t> pos(cnt.begin(), cnt.end() - 1);
    for (int64_t e = 0; e < m; ++e) rows[pos[tgt[e]]++] = src[e];
  }
  std::vector<uint32_t>().swap(src);
  std::vector<int64_t> ucnt(n + 1, 0);
#pragma omp parallel for schedule(dynamic, 1024)
  for (int64_t c = 0; c < n; ++c) {
    uint32_t* b = rows.data() + cnt[c];
    uint32_t* e = rows.data() + cnt[c + 1];
    std::sort(b, e);
    int64_t u = 0;
    for (uint32_t* p = b; p < e; ++p) u += (p == b || p[0] != p[-1]);
    ucnt[c + 1] = u;
  }
  for (int64_t c = 0; c < n; ++c) ucnt[c + 1] += ucnt[c];
  const int64_t nnz = ucnt[n];
  out->nrow = n; out->ncol = n; out->nnz = nnz;
  out->colptr = (int64_t*)malloc(sizeof(int64_t) * (n + 1));
  out->row = (int32_t*)malloc(sizeof(int32_t) * (nnz + 1));
  out->val = (double*)malloc(sizeof(double) * (nnz + 1));
  if (!out->colptr || !out->row || !out->val) { cbg_host_free(out); return CBG_ENOMEM; }
  memcpy(out->colptr, ucnt.data(), sizeof(int64_t) * (n + 1));
#pragma omp parallel for schedule(dynamic, 1024)
  for (int64_t c = 0; c < n; ++c) {
    const uint32_t* b = rows.data() + cnt[c];
    const uint32_t* e = rows.data() + cnt[c + 1];
    int64_t o = ucnt[c];
    for (const uint32_t* p = b; p < e;) {
      const uint32_t* q = p;
      while (q < e && *q == *p) ++q;
      out->row[o] = (int32_t)*p;
      out->val[o] = (double)(q - p);   // multiplicity (SpTuples.cpp:66-115 sums duplicates)
      ++o;
      p = q;
    }
  }
  return CBG_OK;
}

extern "C" void cbg_host_free(cbg_host_csc* m) {
  if (!m) return;
  free(m->colptr); free(m->row); free(m->val);
  memset(m, 0, sizeof(*m));
}
