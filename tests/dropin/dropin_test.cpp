// tests/dropin/dropin_test.cpp -- TEST INFRASTRUCTURE: the C++ drop-in (include/combblas_gpu.h)
// against the reference's own types and kernels, in one process.
//
// Builds SpDCCols<int64_t, T> operands through the reference's SpTuples -> SpDCCols path, runs
// combblas::gpu::LocalSpGEMMHash (libcbgpu) and the reference's combblas::LocalSpGEMMHash (CPU), and
// compares the column-sorted products entry by entry (the reference output is re-sorted with
// SortColBased: its integerSort mis-sorts power-of-two rows).  Also MultiwayMerge and a
// semiring without a device functor (must take the reference CPU path).  The distributed drivers
// (gpu::Mult_AnXBn_Synch / DoubleBuff / Overlap / PSpGEMM, libcbgpu's grid over the SpParMat's MPI
// communicators) are compared block by block with the reference's Mult_AnXBn_Synch on the same
// SpParMat operands; run it under mpirun -np 1 or 4 (square grids, CommGrid.cpp:44-50).
//   usage: dropin_test [--expect-no-gpu]
// Exit 0 = all equal (or, with --expect-no-gpu, the device path threw a device error).
//
// 3D mode (mpirun -np q*q*L):  dropin_test --3d <q> <L> <A.mtx> <C.mtx> <G.mtx>
// restriction (mpirun -np q*q): dropin_test --restrict <q> <A.mtx> <agg.txt>
//   * the split-3D driver of 3DSpGEMM exactly as test_mpipspgemm.cpp:101-153 sets it up (CCGrid, ReadMat
//     unpermuted, SplitMat): gpu::multiply (column and outer/isBT modes) and gpu::SUMMALayer against the
//     reference's multiply / SUMMALayer on the same split pieces, and against controlC (C.mtx = MATLAB A*A);
//   * gpu::Mult_AnXBn_SUMMA3D against the reference's Mult_AnXBn_SUMMA3D (ParFriends.h:2918-3208) on
//     SpParMat3D(A2D, L, colsplit) x SpParMat3D(A2D, L, rowsplit) for A = A.mtx (real values: within
//     1e-12 of max(|c|, sum|a*b|)) and A = G.mtx (integer values: bit-exact), rank piece by rank piece.
#include <mpi.h>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <tuple>
#include <vector>
#include "CombBLAS/CombBLAS.h"
#include "3DSpGEMM/CCGrid.h"
#include "3DSpGEMM/Reductions.h"
#include "3DSpGEMM/Multiplier.h"
#include "3DSpGEMM/SplitMatDist.h"
#include "combblas_gpu.h"
using namespace combblas;

// timers the 3DSpGEMM headers declare extern (3DSpGEMM/Glue.h; test_mpipspgemm.cpp:22-30 defines them)
double comm_bcast, comm_reduce, comp_summa, comp_reduce, comp_result, comp_reduce_layer, comp_split, comp_trans,
    comm_split;

typedef int64_t I;

template <class T>
SpDCCols<I, T>* random_dccols(I m, I n, double density, unsigned seed) {
  std::mt19937_64 g(seed);
  std::uniform_real_distribution<double> u(0.0, 1.0);
  std::vector<std::tuple<I, I, T>> tv;
  for (I j = 0; j < n; ++j)
    for (I i = 0; i < m; ++i)
      if (u(g) < density) tv.emplace_back(i, j, (T)(1 + (g() % 9)));
  std::tuple<I, I, T>* t = new std::tuple<I, I, T>[tv.size()];
  for (size_t k = 0; k < tv.size(); ++k) t[k] = tv[k];
  SpTuples<I, T> tup((int64_t)tv.size(), m, n, t, true);
  return new SpDCCols<I, T>(tup, false);
}

template <class T>
bool same(SpTuples<I, T>* a, SpTuples<I, T>* b, const char* what) {
  a->SortColBased();
  b->SortColBased();
  if (a->getnnz() != b->getnnz()) { printf("%s: nnz %lld vs %lld\n", what, (long long)a->getnnz(), (long long)b->getnnz()); return false; }
  for (I k = 0; k < a->getnnz(); ++k)
    if (a->rowindex(k) != b->rowindex(k) || a->colindex(k) != b->colindex(k) || a->numvalue(k) != b->numvalue(k)) {
      printf("%s: entry %lld differs\n", what, (long long)k);
      return false;
    }
  printf("%s: %lld entries equal\n", what, (long long)a->getnnz());
  return true;
}

// the rank's block of a deterministic global random M x N matrix (same stream on every rank)
template <class T>
SpDCCols<I, T>* random_block(std::shared_ptr<CommGrid> grid, I M, I N, double density, unsigned seed) {
  const int q = grid->GetGridRows(), i = grid->GetRankInProcCol(), j = grid->GetRankInProcRow();
  const I r0 = i * (M / q), r1 = (i == q - 1) ? M : r0 + M / q;
  const I c0 = j * (N / q), c1 = (j == q - 1) ? N : c0 + N / q;
  std::mt19937_64 g(seed);
  std::uniform_real_distribution<double> u(0.0, 1.0);
  std::vector<std::tuple<I, I, T>> tv;
  for (I c = 0; c < N; ++c)
    for (I r = 0; r < M; ++r) {
      const bool on = u(g) < density;
      const T v = (T)(1 + (g() % 9));
      if (on && r >= r0 && r < r1 && c >= c0 && c < c1) tv.emplace_back(r - r0, c - c0, v);
    }
  std::tuple<I, I, T>* t = new std::tuple<I, I, T>[tv.size() > 0 ? tv.size() : 1];
  for (size_t k = 0; k < tv.size(); ++k) t[k] = tv[k];
  SpTuples<I, T> tup((int64_t)tv.size(), r1 - r0, c1 - c0, t, true);
  return new SpDCCols<I, T>(tup, false);
}

// duplicates combined by + (the reference's multi-rank Synch leaves duplicates: SURVEY §0.5)
template <class T>
SpTuples<I, T>* dedup_sum(SpTuples<I, T>* a) {
  a->SortColBased();
  std::vector<std::tuple<I, I, T>> v;
  for (I k = 0; k < a->getnnz(); ++k) {
    if (!v.empty() && std::get<0>(v.back()) == a->rowindex(k) && std::get<1>(v.back()) == a->colindex(k))
      std::get<2>(v.back()) += a->numvalue(k);
    else
      v.emplace_back(a->rowindex(k), a->colindex(k), a->numvalue(k));
  }
  std::tuple<I, I, T>* t = new std::tuple<I, I, T>[v.size() > 0 ? v.size() : 1];
  for (size_t k = 0; k < v.size(); ++k) t[k] = v[k];
  SpTuples<I, T>* r = new SpTuples<I, T>((int64_t)v.size(), a->getnrow(), a->getncol(), t, true);
  delete a;
  return r;
}

template <class T1, class T2>
struct MaxTimesSR {   // no device functor: must run the reference CPU template
  typedef typename promote_trait<T1, T2>::T_promote T_promote;
  static T_promote id() { return 0; }
  static bool returnedSAID() { return false; }
  static MPI_Op mpi_op() { return MPI_MAX; }
  static T_promote add(const T_promote& a, const T_promote& b) { return a > b ? a : b; }
  static T_promote multiply(const T1& a, const T2& b) { return (T_promote)a * (T_promote)b; }
};

// device product vs reference product: identical structure; values within 1e-12 * max(|ref|, scale) where
// `scale` (same structure) holds sum|a*b| per entry, or bit-exact when scale is null
template <class IT, class T>
bool close(SpTuples<IT, T>* d, SpTuples<IT, T>* r, SpTuples<IT, T>* scale, const char* what) {
  d->SortColBased();
  r->SortColBased();
  if (scale) scale->SortColBased();
  if (d->getnnz() != r->getnnz() || (scale && scale->getnnz() != r->getnnz())) {
    printf("%s: nnz %lld vs %lld\n", what, (long long)d->getnnz(), (long long)r->getnnz());
    return false;
  }
  int64_t off = 0;
  for (IT k = 0; k < r->getnnz(); ++k) {
    if (d->rowindex(k) != r->rowindex(k) || d->colindex(k) != r->colindex(k)) {
      printf("%s: entry %lld at (%lld,%lld) vs (%lld,%lld)\n", what, (long long)k, (long long)d->rowindex(k),
             (long long)d->colindex(k), (long long)r->rowindex(k), (long long)r->colindex(k));
      return false;
    }
    const double a = (double)d->numvalue(k), b = (double)r->numvalue(k);
    const double tol = scale ? 1e-12 * std::max(std::fabs(b), (double)scale->numvalue(k)) : 0.0;
    if (std::fabs(a - b) > tol) ++off;
  }
  printf("%s: %lld entries, %lld off\n", what, (long long)r->getnnz(), (long long)off);
  return off == 0;
}

template <class IT, class T>
SpDCCols<IT, T> abs_copy(const SpDCCols<IT, T>& M) {
  SpDCCols<IT, T> c(M);
  c.Apply([](T x) { return (T)std::fabs((double)x); });
  return c;
}

// the split-3D driver (3DSpGEMM) and Mult_AnXBn_SUMMA3D against the reference's own on the same pieces
int run3d(int q, int L, const std::string& fa, const std::string& fc, const std::string& fg) {
  int rc = 0;
  {
    CCGrid CMG(L, q);
    typedef int32_t IT3;
    SpDCCols<IT3, double> splitA, splitB, controlC;
    {
      std::shared_ptr<CommGrid> layerGrid(new CommGrid(CMG.layerWorld, 0, 0));
      FullyDistVec<IT3, IT3> p(layerGrid);
      SpDCCols<IT3, double>* A = ReadMat<double>(fa, CMG, false, p);
      SpDCCols<IT3, double>* B = ReadMat<double>(fa, CMG, false, p);
      SpDCCols<IT3, double>* C = ReadMat<double>(fc, CMG, false, p);
      SplitMat(CMG, A, splitA, false);
      SplitMat(CMG, B, splitB, true);
      SplitMat(CMG, C, controlC, false);
    }
    SpDCCols<IT3, double> absA = abs_copy(splitA), absB = abs_copy(splitB);
    SpDCCols<IT3, double>* S = multiply(absA, absB, CMG, false, true);   // sum|a*b| per entry (reference)
    SpDCCols<IT3, double>* R = multiply(splitA, splitB, CMG, false, true);
    SpDCCols<IT3, double>* D = gpu::multiply(splitA, splitB, CMG, false, true);
    {
      const cbg_grid_info& gi = gpu::last_grid_info();
      printf("GRID rccl=%d world=%d row=%d col=%d fiber=%d\n", gi.rccl, gi.ranks[CBG_GROUP_WORLD],
             gi.ranks[CBG_GROUP_ROW], gi.ranks[CBG_GROUP_COL], gi.ranks[CBG_GROUP_FIBER]);
    }
    SpTuples<IT3, double> st(*S);
    {
      SpTuples<IT3, double> dt(*D), rt(*R), ct(controlC), s2(st);
      if (!close(&dt, &rt, &st, "gpu::multiply vs reference multiply")) rc = 1;
      if (!close(&dt, &ct, &s2, "gpu::multiply vs MATLAB C.mtx (controlC)")) rc = 1;
    }
    SpDCCols<IT3, double> splitBT(splitB);
    splitBT.Transpose();   // "outer": B held locally transposed (test_mpipspgemm.cpp:101-107)
    SpDCCols<IT3, double>* DO = gpu::multiply(splitA, splitBT, CMG, true, false);
    {
      SpTuples<IT3, double> dt(*DO), rt(*R);
      if (!close(&dt, &rt, &st, "gpu::multiply isBT vs reference multiply")) rc = 1;
    }
    std::vector<SpTuples<IT3, double>*> rl, dl, sl;
    SUMMALayer(splitA, splitB, rl, CMG, false, true);
    gpu::SUMMALayer(splitA, splitB, dl, CMG, false, true);
    SUMMALayer(absA, absB, sl, CMG, false, true);
    if (rl.size() != dl.size()) { printf("SUMMALayer: %zu vs %zu stage products\n", dl.size(), rl.size()); rc = 1; }
    for (size_t k = 0; k < std::min(rl.size(), dl.size()); ++k) {
      char what[64];
      snprintf(what, sizeof what, "gpu::SUMMALayer stage %zu", k);
      if (!close(dl[k], rl[k], sl[k], what)) rc = 1;
    }
    for (auto* t : rl) delete t;
    for (auto* t : dl) delete t;
    for (auto* t : sl) delete t;
    delete S; delete R; delete D; delete DO;
  }
  // Mult_AnXBn_SUMMA3D on SpParMat3D(A2D, L, colsplit) x SpParMat3D(A2D, L, rowsplit).  The reference builds an
  // SpParMat3D from a 2D SpParMat on a square CommGrid of all ranks (CommGrid.cpp:37-76), so this part runs
  // where the world is a square (4 ranks: 2x2x1 and 1x1x4); 2 and 8 ranks cover the split-3D driver only.
  const int world = q * q * L;
  const int side = (int)std::lround(std::sqrt((double)world));
  for (int f = 0; f < 2 && side * side == world; ++f) {
    typedef SpDCCols<I, double> DCC;
    typedef SpParMat<I, double, DCC> PM;
    typedef SpParMat3D<I, double, DCC> PM3;
    typedef PlusTimesSRing<double, double> PT;
    const std::string& file = f == 0 ? fa : fg;
    std::shared_ptr<CommGrid> grid(new CommGrid(MPI_COMM_WORLD, 0, 0));
    PM A(grid), B(grid);
    A.ParallelReadMM(file, true, maximum<double>());
    B.ParallelReadMM(file, true, maximum<double>());
    PM3 A3(A, L, true, false), B3(B, L, false, false);
    PM3 R = Mult_AnXBn_SUMMA3D<PT, double, DCC>(A3, B3);
    PM3 D = gpu::Mult_AnXBn_SUMMA3D<PT, double, DCC>(A3, B3);
    SpTuples<I, double> rt(*R.seqptr()), dt(*D.seqptr());
    if (f == 0) {
      PM Aa(A), Ba(B);
      Aa.Apply([](double x) { return std::fabs(x); });
      Ba.Apply([](double x) { return std::fabs(x); });
      PM3 Aa3(Aa, L, true, false), Ba3(Ba, L, false, false);
      PM3 S3 = Mult_AnXBn_SUMMA3D<PT, double, DCC>(Aa3, Ba3);
      SpTuples<I, double> s3(*S3.seqptr());
      if (!close(&dt, &rt, &s3, "gpu::Mult_AnXBn_SUMMA3D vs reference (A.mtx)")) rc = 1;
    } else {
      if (!close(&dt, &rt, (SpTuples<I, double>*)nullptr, "gpu::Mult_AnXBn_SUMMA3D vs reference (G.mtx, exact)")) rc = 1;
    }
  }
  int any = 0;
  MPI_Allreduce(&rc, &any, 1, MPI_INT, MPI_MAX, MPI_COMM_WORLD);
  return any;
}

// gpu::RestrictionOp (3DSpGEMM/RestrictionOp.h:196-291) on a q x q layer: every rank's R and R^T blocks against the
// reference's one-rank R (aggregate of every vertex, from oracle/_ref/refrestrict via tests/golden/restriction.npz)
int run_restrict(int q, const std::string& fa, const std::string& fagg) {
  int rc = 0;
  typedef SpDCCols<I, double> DCC;
  CCGrid CMG(1, q);
  std::shared_ptr<CommGrid> lg(new CommGrid(CMG.layerWorld, 0, 0));
  SpParMat<I, double, DCC> A(lg);
  A.ParallelReadMM(fa, true, maximum<double>());
  DCC* local = new DCC(*A.seqptr());
  DCC *R = nullptr, *RT = nullptr;
  gpu::RestrictionOp(CMG, local, R, RT);
  std::vector<int64_t> agg;
  {
    FILE* f = fopen(fagg.c_str(), "r");
    long long x;
    while (f && fscanf(f, "%lld", &x) == 1) agg.push_back(x);
    if (f) fclose(f);
  }
  const int64_t M = (int64_t)agg.size(), nagg = agg.empty() ? 0 : *std::max_element(agg.begin(), agg.end()) + 1;
  int lr = 0;
  MPI_Comm_rank(CMG.layerWorld, &lr);
  const int bi = lr / q, bj = lr % q;
  auto blk = [q](int64_t len, int b, int64_t* lo, int64_t* hi) {
    *lo = (len / q) * b;
    *hi = b == q - 1 ? len : (len / q) * (b + 1);
  };
  int64_t r0, r1, c0, c1, t0, t1, u0, u1;
  blk(M, bi, &r0, &r1);
  blk(nagg, bj, &c0, &c1);
  blk(nagg, bi, &t0, &t1);
  blk(M, bj, &u0, &u1);
  if (R->getnrow() != r1 - r0 || R->getncol() != c1 - c0 || RT->getnrow() != t1 - t0 || RT->getncol() != u1 - u0) {
    printf("restrict: block shapes differ\n");
    rc = 1;
  }
  int64_t want_r = 0, want_t = 0;
  for (int64_t v = r0; v < r1; ++v) want_r += agg[(size_t)v] >= c0 && agg[(size_t)v] < c1;
  for (int64_t v = u0; v < u1; ++v) want_t += agg[(size_t)v] >= t0 && agg[(size_t)v] < t1;
  SpTuples<I, double> TR(*R), TT(*RT);
  int64_t off = 0;
  for (int64_t k = 0; k < TR.getnnz(); ++k)
    off += agg[(size_t)(TR.rowindex(k) + r0)] != TR.colindex(k) + c0 || TR.numvalue(k) != 1.0;
  for (int64_t k = 0; k < TT.getnnz(); ++k) off += agg[(size_t)(TT.colindex(k) + u0)] != TT.rowindex(k) + t0;
  if (off || TR.getnnz() != want_r || TT.getnnz() != want_t) {
    printf("restrict: rank %d: %lld entries off, nnz R %lld (want %lld), R^T %lld (want %lld)\n", lr, (long long)off,
           (long long)TR.getnnz(), (long long)want_r, (long long)TT.getnnz(), (long long)want_t);
    rc = 1;
  } else {
    printf("gpu::RestrictionOp rank %d: R block %lld entries, R^T block %lld, equal to the reference's R\n", lr,
           (long long)TR.getnnz(), (long long)TT.getnnz());
  }
  delete R;
  delete RT;
  delete local;
  int any = 0;
  MPI_Allreduce(&rc, &any, 1, MPI_INT, MPI_MAX, MPI_COMM_WORLD);
  return any;
}

int main(int argc, char** argv) {
  MPI_Init(&argc, &argv);
  if (argc == 5 && std::string(argv[1]) == "--restrict") {
    int rc = 1;
    try {
      rc = run_restrict(atoi(argv[2]), argv[3], argv[4]);
    } catch (std::exception& e) {
      printf("restrict: %s\n", e.what());
    }
    MPI_Finalize();
    printf(rc == 0 ? "DROPINR OK\n" : "DROPINR FAILED\n");
    return rc;
  }
  if (argc == 7 && std::string(argv[1]) == "--3d") {
    int rc = 1;
    try {
      rc = run3d(atoi(argv[2]), atoi(argv[3]), argv[4], argv[5], argv[6]);
    } catch (std::exception& e) {
      printf("3d: %s\n", e.what());
    }
    MPI_Finalize();
    printf(rc == 0 ? "DROPIN3D OK\n" : "DROPIN3D FAILED\n");
    return rc;
  }
  const bool expect_no_gpu = argc > 1 && std::string(argv[1]) == "--expect-no-gpu";
  int rc = 0;
  {
    auto* A = random_dccols<double>(300, 250, 0.05, 1);
    auto* B = random_dccols<double>(250, 200, 0.05, 2);
    typedef PlusTimesSRing<double, double> PT;
    SpTuples<I, double>* ref = LocalSpGEMMHash<PT, double>(*A, *B, false, false, true);
    SpTuples<I, double>* dev = nullptr;
    try {
      dev = gpu::LocalSpGEMMHash<PT, double>(*A, *B, false, false, true);
    } catch (std::exception& e) {
      printf("device path: %s\n", e.what());
      MPI_Finalize();
      return expect_no_gpu ? 0 : 2;
    }
    if (expect_no_gpu) { printf("expected no GPU but the device path ran\n"); rc = 3; }
    if (!same(dev, ref, "PlusTimes<double>")) rc = 1;

    auto* Ai = random_dccols<int64_t>(120, 90, 0.1, 3);
    auto* Bi = random_dccols<int64_t>(90, 110, 0.1, 4);
    typedef MinPlusSRing<int64_t, int64_t> MP;
    SpTuples<I, int64_t>* ri = LocalSpGEMMHash<MP, int64_t>(*Ai, *Bi, false, false, true);
    SpTuples<I, int64_t>* di = gpu::LocalSpGEMMHash<MP, int64_t>(*Ai, *Bi, false, false, true);
    if (!same(di, ri, "MinPlus<int64>")) rc = 1;

    // bool-valued product (bool values are staged as bytes on the host side of the drop-in)
    auto* Ab = random_dccols<bool>(140, 100, 0.08, 6);
    auto* Bb = random_dccols<bool>(100, 120, 0.08, 7);
    typedef PlusTimesSRing<bool, bool> PTB;
    SpTuples<I, bool>* rb = LocalSpGEMMHash<PTB, bool>(*Ab, *Bb, false, false, true);
    SpTuples<I, bool>* db = gpu::LocalSpGEMMHash<PTB, bool>(*Ab, *Bb, false, false, true);
    if (!same(db, rb, "PlusTimes<bool>")) rc = 1;
    std::vector<SpTuples<I, bool>*> lb1 = {new SpTuples<I, bool>(*rb), new SpTuples<I, bool>(*db)};
    std::vector<SpTuples<I, bool>*> lb2 = {new SpTuples<I, bool>(*rb), new SpTuples<I, bool>(*db)};
    SpTuples<I, bool>* mbr = MultiwayMerge<PTB>(lb1, (I)140, (I)120, true);
    SpTuples<I, bool>* mbd = gpu::MultiwayMerge<PTB>(lb2, (I)140, (I)120, true);
    if (!same(mbd, mbr, "MultiwayMerge<bool>")) rc = 1;
    delete rb; delete db; delete mbr; delete mbd; delete Ab; delete Bb;

    typedef MaxTimesSR<int64_t, int64_t> MT;   // CPU fallback inside the drop-in
    SpTuples<I, int64_t>* rc1 = LocalSpGEMMHash<MT, int64_t>(*Ai, *Bi, false, false, true);
    SpTuples<I, int64_t>* dc1 = gpu::LocalSpGEMMHash<MT, int64_t>(*Ai, *Bi, false, false, true);
    if (!same(dc1, rc1, "custom semiring (CPU template)")) rc = 1;

    // MultiwayMerge of two products of the same shape
    std::vector<SpTuples<I, double>*> l1 = {new SpTuples<I, double>(*ref), new SpTuples<I, double>(*dev)};
    std::vector<SpTuples<I, double>*> l2 = {new SpTuples<I, double>(*ref), new SpTuples<I, double>(*dev)};
    SpTuples<I, double>* mr = MultiwayMerge<PT>(l1, (I)300, (I)200, true);
    SpTuples<I, double>* md = gpu::MultiwayMerge<PT>(l2, (I)300, (I)200, true);
    if (!same(md, mr, "MultiwayMerge")) rc = 1;

    const int64_t f = gpu::EstimateLocalFLOP<PT>(*A, *B);
    int64_t fr = 0;
    { Arr<I, double> a = B->GetArrays(); (void)a; }
    fr = EstimateLocalFLOP<PT>(*A, *B, false, false);
    printf("EstimateLocalFLOP device %lld reference %lld\n", (long long)f, (long long)fr);
    if (f != fr) rc = 1;
    delete ref; delete dev; delete ri; delete di; delete rc1; delete dc1; delete mr; delete md;
    delete A; delete B; delete Ai; delete Bi;

    // MCLPruneRecoverySelect on a 1-rank SpParMat: reference (CPU, ParFriends.h:185-353) vs drop-in
    {
      typedef SpDCCols<I, double> DCC;
      typedef SpParMat<I, double, DCC> PM;
      std::shared_ptr<CommGrid> grid(new CommGrid(MPI_COMM_WORLD, 0, 0));
      auto* P = random_dccols<double>(300, 300, 0.08, 5);
      SpTuples<I, double>* sq = LocalSpGEMMHash<PT, double>(*P, *P, false, false, true);
      sq->SortColBased();
      for (I k = 0; k < sq->getnnz(); ++k) std::get<2>(sq->tuples[k]) = 1.0 / (1.0 + std::get<2>(sq->tuples[k]));
      const double params[3][4] = {{1e-4, 1100, 1400, 0.9}, {0.05, 10, 15, 0.9}, {0.3, 5, 8, 0.99}};
      for (auto& p : params) {
        PM R(new DCC(*sq, false), grid), D(new DCC(*sq, false), grid);
        combblas::MCLPruneRecoverySelect(R, p[0], (I)p[1], (I)p[2], p[3], 1);
        gpu::MCLPruneRecoverySelect(D, p[0], (I)p[1], (I)p[2], p[3], 1);
        SpTuples<I, double>* a = new SpTuples<I, double>(R.seq());
        SpTuples<I, double>* b = new SpTuples<I, double>(D.seq());
        if (!same(b, a, "MCLPruneRecoverySelect")) rc = 1;
        delete a; delete b;
      }
      delete sq; delete P;
    }
    // distributed drivers on the SpParMat's grid, block by block against the reference's Synch
    {
      typedef SpDCCols<I, int64_t> DI;
      typedef SpParMat<I, int64_t, DI> PMI;
      typedef PlusTimesSRing<int64_t, int64_t> PTI;
      std::shared_ptr<CommGrid> grid(new CommGrid(MPI_COMM_WORLD, 0, 0));
      PMI A(random_block<int64_t>(grid, 420, 380, 0.05, 11), grid);
      PMI B(random_block<int64_t>(grid, 380, 350, 0.05, 12), grid);
      PMI R = combblas::Mult_AnXBn_Synch<PTI, int64_t, DI>(A, B);
      SpTuples<I, int64_t>* rt = dedup_sum(new SpTuples<I, int64_t>(R.seq()));
      const char* names[4] = {"gpu::Mult_AnXBn_Synch", "gpu::Mult_AnXBn_DoubleBuff", "gpu::Mult_AnXBn_Overlap",
                              "gpu::PSpGEMM"};
      for (int d = 0; d < 4; ++d) {
        PMI D = d == 0 ? gpu::Mult_AnXBn_Synch<PTI, int64_t, DI>(A, B)
              : d == 1 ? gpu::Mult_AnXBn_DoubleBuff<PTI, int64_t, DI>(A, B)
              : d == 2 ? gpu::Mult_AnXBn_Overlap<PTI, int64_t, DI>(A, B)
                       : gpu::PSpGEMM<PTI>(A, B);
        SpTuples<I, int64_t>* dt = new SpTuples<I, int64_t>(D.seq());
        SpTuples<I, int64_t>* rc2 = new SpTuples<I, int64_t>(*rt);
        if (!same(dt, rc2, names[d])) rc = 1;
        delete dt; delete rc2;
      }
      delete rt;
      // the grid is set up once per CommGrid and reused (HipMCL calls the driver every iteration): ten back-to-back
      // Mult_AnXBn_Synch calls, per-call wall time, and the process's grid setups before / after them
      {
        const int before = gpu::grid_creations();
        double tmin = 1e30, tmax = 0, tsum = 0;
        for (int it = 0; it < 10; ++it) {
          MPI_Barrier(MPI_COMM_WORLD);
          const double t0 = MPI_Wtime();
          PMI D = gpu::Mult_AnXBn_Synch<PTI, int64_t, DI>(A, B);
          MPI_Barrier(MPI_COMM_WORLD);
          const double t = MPI_Wtime() - t0;
          tmin = std::min(tmin, t); tmax = std::max(tmax, t); tsum += t;
        }
        printf("REPEAT calls=10 setups_before=%d setups_after=%d ms_min=%.3f ms_mean=%.3f ms_max=%.3f\n", before,
               gpu::grid_creations(), 1e3 * tmin, 1e2 * tsum, 1e3 * tmax);
        if (gpu::grid_creations() != before) rc = 1;
      }
      const cbg_grid_info& gi = gpu::last_grid_info();   // the grid the drivers ran over
      printf("GRID rccl=%d world=%d row=%d col=%d fiber=%d\n", gi.rccl, gi.ranks[CBG_GROUP_WORLD],
             gi.ranks[CBG_GROUP_ROW], gi.ranks[CBG_GROUP_COL], gi.ranks[CBG_GROUP_FIBER]);
      int bad = rc, any = 0;
      MPI_Allreduce(&bad, &any, 1, MPI_INT, MPI_MAX, MPI_COMM_WORLD);
      rc = any;
    }
  }
  MPI_Finalize();
  printf(rc == 0 ? "DROPIN OK\n" : "DROPIN FAILED\n");
  return rc;
}
