// rmat.cpp -- the reference's Graph500 Kronecker (R-MAT) matrix built on the host (no GPU needed).
//
// The edge stream is the reference's own (kron.hpp: RefGen21.h:102-318, DistEdgeList.cpp:223-280,
// packed path); the matrix build follows SpParMat(DistEdgeList, removeloops=false)
// (SpParMat.cpp:3082-3196) and the duplicate-summing SpTuples constructor (SpTuples.cpp:66-115):
// edge (v0, v1) -> A(v0, v1), duplicates summed into the value = multiplicity (f64), loops kept.
// The device build of the same matrix (and of any block of it) is cbg_rmat_block in kron.hip.
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include <algorithm>
#include "cbgpu.h"
#include "kron.hpp"

extern "C" cbg_status cbg_rmat_host(int32_t scale, int32_t edgefactor, uint64_t seed, cbg_host_csc* out) {
  if (!out || scale < 1 || scale > 31 || edgefactor < 1) return CBG_EINVAL;
  memset(out, 0, sizeof(*out));
  const int64_t n = 1ll << scale;
  const int64_t m = (int64_t)edgefactor << scale;
  using namespace cbg::kron;
  if (((uint64_t)m >> (8 * kSkipBytes)) != 0) return CBG_EUNSUP;
  std::vector<Mat> tab(kSkipBytes * 256);
  const Params p = make_params(seed, tab.data());
  std::vector<uint32_t> src(m), tgt(m);
  const int64_t run = 64;   // one table jump per run of edges, then one A^(2^64) step per edge
#pragma omp parallel for schedule(static)
  for (int64_t r0 = 0; r0 < m; r0 += run) {
    State z = p.base;
    for (uint64_t ei = (uint64_t)r0, i = 0; ei; ++i, ei >>= 8)
      if (ei & 0xFF) apply(tab[i * 256 + (ei & 0xFF)], z);
    for (int64_t e = r0; e < std::min(m, r0 + run); ++e) {
      int64_t s0, t0;
      edge_unscrambled(z, scale, &s0, &t0);
      src[e] = (uint32_t)scramble(s0, scale, p.val0, p.val1);
      tgt[e] = (uint32_t)scramble(t0, scale, p.val0, p.val1);
      apply(tab[1], z);
    }
  }
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
