// kron.hip -- Graph500 Kronecker (R-MAT) input built on the device, one block per rank.
//
// Replaces the reference's input pipeline for its R-MAT runs:
//   DistEdgeList::GenGraph500Data(packed)  include/CombBLAS/DistEdgeList.cpp:223-280
//   RefGen21::generate_kronecker_range     include/CombBLAS/RefGen21.h:242-262 (edge stream, kron.hpp)
//   SpParMat(DistEdgeList&, removeloops)   include/CombBLAS/SpParMat.cpp:3082-3196 (edge owner routing)
//   SpTuples(edges) + SpDCCols(SpTuples)   include/CombBLAS/SpTuples.cpp:66-115, SpDCCols.cpp:109-184
//                                          (duplicate edges summed into the value = multiplicity)
// The reference generates 1/p of the edges per rank and routes each edge to its owner with an
// all-to-all; here every rank replays the whole counter-based stream on its GPU and keeps the edges of
// its own block, so no collective is needed (the stream costs ~1 ns per edge, far below the transfer).
//
// Device pipeline for block [r0, r1) x [c0, c1):
//   k_kron_edges   each lane generates a run of edges (one table jump, then one A^(2^64) step per
//                  edge), keeps the in-block ones: (row, col) appended with a wave-aggregated atomic,
//                  column histogram;
//   scan           column pointers of the raw (duplicated, unsorted) block;
//   k_kron_scatter rows into their columns;
//   dedup_columns  I * Araw, the local hash SpGEMM with a pattern identity (spgemm_host.hpp):
//                  duplicates of (row, col) sum to the multiplicity and every column comes out
//                  row-sorted -- the SpTuples duplicate-summing constructor as one device product.
#include "spgemm_host.hpp"
#include "kron.hpp"

namespace {
using namespace cbg::kron;

constexpr int kEdgesPerLane = 8;

__global__ void __launch_bounds__(256) k_kron_edges(Params p, const Mat* __restrict__ tab, int lgN, uint64_t e0,
                                                    uint64_t e1, int64_t r0, int64_t r1, int64_t c0, int64_t c1,
                                                    uint2* __restrict__ out, unsigned long long* __restrict__ nout,
                                                    unsigned long long* __restrict__ colcnt) {
  const Mat step = tab[1];   // A^(2^64): edge ei -> ei + 1
  const uint64_t nrun = (e1 - e0 + kEdgesPerLane - 1) / kEdgesPerLane;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  // every lane of a wave runs the loop the same number of times (ballots below need the whole wave)
  const uint64_t iters = (nrun + stride - 1) / stride;
  for (uint64_t it = 0; it < iters; ++it) {
    const uint64_t run = it * stride + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const uint64_t first = e0 + run * kEdgesPerLane;
    State z = p.base;
    if (run < nrun) {
      uint64_t ei = first;
      for (int i = 0; ei; ++i, ei >>= 8) {
        const uint32_t k = (uint32_t)(ei & 0xFF);
        if (k) apply(tab[i * 256 + k], z);
      }
    }
    for (int e = 0; e < kEdgesPerLane; ++e) {
      const uint64_t ei = first + e;
      bool keep = false;
      int64_t src = 0, tgt = 0;
      if (run < nrun && ei < e1) {
        edge_unscrambled(z, lgN, &src, &tgt);
        src = scramble(src, lgN, p.val0, p.val1);
        tgt = scramble(tgt, lgN, p.val0, p.val1);
        keep = src >= r0 && src < r1 && tgt >= c0 && tgt < c1;   // owner of (src, tgt): row src, column tgt
        if (e + 1 < kEdgesPerLane) apply(step, z);
      }
      const uint64_t mask = __ballot(keep);
      if (mask == 0) continue;
      const int lane = __lane_id();
      const int leader = __ffsll((unsigned long long)mask) - 1;
      unsigned long long base = 0;
      if (lane == leader) base = atomicAdd(nout, (unsigned long long)__popcll(mask));
      base = __shfl(base, leader);
      if (keep) {
        const unsigned long long below = mask & ((1ull << lane) - 1);
        out[base + __popcll(below)] = make_uint2((uint32_t)(src - r0), (uint32_t)(tgt - c0));
        atomicAdd(&colcnt[tgt - c0], 1ull);
      }
    }
  }
}

__global__ void k_kron_scatter(uint64_t n, const uint2* __restrict__ e, unsigned long long* __restrict__ cursor,
                               int32_t* __restrict__ rows) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint2 rc = e[i];
    rows[atomicAdd(&cursor[rc.y], 1ull)] = (int32_t)rc.x;
  }
}

}  // namespace

extern "C" cbg_status cbg_rmat_block(cbg_ctx* ctx, int32_t scale, int32_t edgefactor, uint64_t seed, int64_t r0,
                                     int64_t r1, int64_t c0, int64_t c1, cbg_csc_result* out) {
  if (!ctx || !out || scale < 1 || scale > 31 || edgefactor < 1) return CBG_EINVAL;
  const int64_t n = 1ll << scale;
  if (r0 < 0 || r1 < r0 || r1 > n || c0 < 0 || c1 < c0 || c1 > n) return CBG_EDIM;
  const int64_t nr = r1 - r0, nc = c1 - c0;
  const uint64_t m = (uint64_t)edgefactor << scale;
  if ((m >> (8 * kSkipBytes)) != 0) return CBG_EUNSUP;
  HIPCHK(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  std::vector<Mat> tab(kSkipBytes * 256);
  const Params p = make_params(seed, tab.data());

  DevBuf dtab, edges, cnt, rows;
  HIPCHK(dtab.reserve(sizeof(Mat) * tab.size()));
  HIPCHK(hipMemcpyAsync(dtab.p, tab.data(), sizeof(Mat) * tab.size(), hipMemcpyHostToDevice, st));
  // in-block edges: the whole stream for a full block, about m * (nr/n) * (nc/n) * skew otherwise;
  // size for the whole stream (8 B per edge) -- 0.5 GB at scale 22
  HIPCHK(edges.reserve(sizeof(uint2) * (m + 1)));
  HIPCHK(cnt.reserve(sizeof(unsigned long long) * (2 * (nc + 1) + 2)));
  unsigned long long* colcnt = cnt.as<unsigned long long>();
  unsigned long long* cursor = colcnt + (nc + 1);
  unsigned long long* nout = cursor + (nc + 1);
  HIPCHK(hipMemsetAsync(cnt.p, 0, sizeof(unsigned long long) * (2 * (nc + 1) + 2), st));
  const uint64_t nrun = (m + kEdgesPerLane - 1) / kEdgesPerLane;
  const int grid = (int)std::min<uint64_t>((nrun + 255) / 256, 8192);
  k_kron_edges<<<grid, 256, 0, st>>>(p, dtab.as<Mat>(), scale, 0, m, r0, r1, c0, c1, edges.as<uint2>(), nout, colcnt);
  HIPCHK(hipGetLastError());
  // column pointers of the raw block (int64 scan of the histogram; ull and int64 share the layout)
  DevBuf tiles, rawcp, scal;
  const int64_t ntiles = (nc + kScanTile - 1) / kScanTile;
  HIPCHK(tiles.reserve(sizeof(int64_t) * (ntiles + 1)));
  HIPCHK(rawcp.reserve(sizeof(int64_t) * (nc + 1)));
  HIPCHK(scal.reserve(64));
  if (nc > 0) {
    k_scan_tiles<<<(int)ntiles, 256, 0, st>>>(nc, (const int64_t*)colcnt, tiles.as<int64_t>());
    k_scan_sums<<<1, 1024, 0, st>>>(ntiles, tiles.as<int64_t>(), scal.as<int64_t>());
    k_scan_apply<<<(int)ntiles, 256, 0, st>>>(nc, (const int64_t*)colcnt, tiles.as<int64_t>(), rawcp.as<int64_t>());
    HIPCHK(hipMemcpyAsync(cursor, rawcp.p, sizeof(int64_t) * nc, hipMemcpyDeviceToDevice, st));
  } else {
    HIPCHK(hipMemsetAsync(rawcp.p, 0, sizeof(int64_t), st));
  }
  unsigned long long nraw = 0;
  HIPCHK(hipMemcpyAsync(&nraw, nout, sizeof(nraw), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  HIPCHK(rows.reserve(sizeof(int32_t) * (nraw + 1)));
  if (nraw)
    k_kron_scatter<<<(int)grid_for((int64_t)nraw, 256, kMaxGrid), 256, 0, st>>>(nraw, edges.as<uint2>(), cursor,
                                                                                rows.as<int32_t>());
  // sum duplicates + row-sort every column (the SpTuples duplicate-summing constructor)
  cbg_status s = dedup_columns(ctx, nr, nc, (int64_t)nraw, rawcp.as<int64_t>(), rows.as<int32_t>(), nullptr, out);
  HIPCHK(hipStreamSynchronize(st));   // scratch above is released on return
  if (s == CBG_OK) out->multiplies = 0;
  return s;
}

extern "C" cbg_status cbg_generate_rmat(cbg_ctx* ctx, int32_t scale, int32_t edgefactor, uint64_t seed,
                                        cbg_csc_result* A) {
  if (scale < 1 || scale > 31) return CBG_EINVAL;
  const int64_t n = 1ll << scale;
  return cbg_rmat_block(ctx, scale, edgefactor, seed, 0, n, 0, n, A);
}
