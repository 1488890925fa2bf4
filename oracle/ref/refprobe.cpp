// oracle/ref/refprobe.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never measured).
//
// Golden-vector generator that drives the *reference* CombBLAS SpGEMM path, compiled
// from the reference's own headers where they lie under /root/reference (see
// oracle/ref/Makefile; output binary goes to oracle/_ref/, which is git-ignored).
// It exists so that tests/golden/ fixtures are outputs of the reference itself,
// not of our restatement.  Reference entry points exercised:
//   LocalSpGEMMHash  include/CombBLAS/mtSpGEMM.h:465-661
//   LocalSpGEMM      include/CombBLAS/mtSpGEMM.h:73-202   (heap)
//   LocalHybridSpGEMM include/CombBLAS/mtSpGEMM.h:212-463
//   EstimateLocalFLOP include/CombBLAS/mtSpGEMM.h:667-694
//   Mult_AnXBn_Synch include/CombBLAS/ParFriends.h:1004-1108
//   DistEdgeList::GenGraph500Data include/CombBLAS/DistEdgeList.cpp:223-280
//   SpParMat::ParallelReadMM include/CombBLAS/SpParMat.cpp:3922
//   MCLPruneRecoverySelect include/CombBLAS/ParFriends.h:185-353 (kselectVersion 1)
//   MemEfficientSpGEMM include/CombBLAS/ParFriends.h:449-730 (hash kernel, phases)
//   MultiwayMerge / MultiwayMergeHash include/CombBLAS/MultiwayMerge.h:411-526, 536-684 (k lists)
// Because of the reference's integerSort off-by-one every product is
// re-sorted column-major with SpTuples::SortColBased before it is written, so
// fixtures hold the mathematically defined product (rows ascending per column).
//
// Binary matrix format ("CBM1", little endian), shared with tests/golden/make_golden.py:
//   char magic[4]="CBM1"; int32 valtype (0=f64,1=i64,2=bool-as-u8);
//   int64 nrow, ncol, nnz; int64 colptr[ncol+1]; int64 row[nnz]; val[nnz]
#include <mpi.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <tuple>
#include "CombBLAS/CombBLAS.h"
using namespace combblas;

typedef int64_t I;

template <class NT> struct VT;
template <> struct VT<double>  { enum { code = 0 }; };
template <> struct VT<int64_t> { enum { code = 1 }; };
template <> struct VT<bool>    { enum { code = 2 }; };

struct RawCsc {
  int32_t vt = 0; I nrow = 0, ncol = 0, nnz = 0;
  std::vector<I> cp, ir; std::vector<double> vd; std::vector<int64_t> vi; std::vector<uint8_t> vb;
};

static RawCsc read_bin(const char* path) {
  RawCsc M; FILE* f = fopen(path, "rb"); if (!f) { perror(path); exit(2); }
  char mg[4]; if (fread(mg, 1, 4, f) != 4 || memcmp(mg, "CBM1", 4)) { fprintf(stderr, "bad magic %s\n", path); exit(2); }
  fread(&M.vt, 4, 1, f); fread(&M.nrow, 8, 1, f); fread(&M.ncol, 8, 1, f); fread(&M.nnz, 8, 1, f);
  M.cp.resize(M.ncol + 1); M.ir.resize(M.nnz);
  fread(M.cp.data(), 8, M.ncol + 1, f); fread(M.ir.data(), 8, M.nnz, f);
  if (M.vt == 0) { M.vd.resize(M.nnz); fread(M.vd.data(), 8, M.nnz, f); }
  else if (M.vt == 1) { M.vi.resize(M.nnz); fread(M.vi.data(), 8, M.nnz, f); }
  else { M.vb.resize(M.nnz); fread(M.vb.data(), 1, M.nnz, f); }
  fclose(f); return M;
}

template <class NT> static NT getv(const RawCsc& M, I k) {
  if (M.vt == 0) return (NT)M.vd[k]; if (M.vt == 1) return (NT)M.vi[k]; return (NT)M.vb[k];
}

template <class NT> static SpDCCols<I, NT>* to_dcc(const RawCsc& M) {
  std::tuple<I, I, NT>* t = new std::tuple<I, I, NT>[M.nnz > 0 ? M.nnz : 1];
  I p = 0;
  for (I c = 0; c < M.ncol; ++c)
    for (I k = M.cp[c]; k < M.cp[c + 1]; ++k) t[p++] = std::make_tuple(M.ir[k], c, getv<NT>(M, k));
  SpTuples<I, NT> T(M.nnz, M.nrow, M.ncol, t, true, false);   // takes ownership
  return new SpDCCols<I, NT>(T, false);
}

template <class NT> static void write_tuples(const char* path, SpTuples<I, NT>& T, I nrow, I ncol) {
  T.SortColBased();   // ColLexiCompare, Compare.h:95-108 (repairs integerSort mis-sorts)
  I nnz = T.getnnz();
  std::vector<I> cp(ncol + 1, 0);
  for (I k = 0; k < nnz; ++k) cp[T.colindex(k) + 1]++;
  for (I c = 0; c < ncol; ++c) cp[c + 1] += cp[c];
  FILE* f = fopen(path, "wb"); fwrite("CBM1", 1, 4, f);
  int32_t vt = VT<NT>::code; fwrite(&vt, 4, 1, f);
  fwrite(&nrow, 8, 1, f); fwrite(&ncol, 8, 1, f); fwrite(&nnz, 8, 1, f);
  fwrite(cp.data(), 8, ncol + 1, f);
  for (I k = 0; k < nnz; ++k) { I r = T.rowindex(k); fwrite(&r, 8, 1, f); }
  for (I k = 0; k < nnz; ++k) {
    if (vt == 2) { uint8_t b = T.numvalue(k) ? 1 : 0; fwrite(&b, 1, 1, f); }
    else { NT v = T.numvalue(k); fwrite(&v, sizeof(NT), 1, f); }
  }
  fclose(f);
}

template <class NT> static void write_dcc(const char* path, SpDCCols<I, NT>& D) {
  SpTuples<I, NT> T(D);
  write_tuples<NT>(path, T, D.getnrow(), D.getncol());
}

// Counts "duplicates": adjacent equal (row,col) after sorting -- the Mult_AnXBn_Synch
// multi-rank bug of SURVEY §0.5 shows up here; at 1 rank it must be zero.
template <class NT> static long count_dups(SpTuples<I, NT>& T) {
  T.SortColBased(); long d = 0;
  for (I k = 1; k < T.getnnz(); ++k) if (T.rowindex(k) == T.rowindex(k - 1) && T.colindex(k) == T.colindex(k - 1)) ++d;
  return d;
}

template <class SR, class NTO, class NT1, class NT2>
static int run_mult(const char* kernel, const RawCsc& RA, const RawCsc& RB, const char* out) {
  SpDCCols<I, NT1>* A = to_dcc<NT1>(RA);
  SpDCCols<I, NT2>* B = to_dcc<NT2>(RB);
  I flops = (A->getnnz() && B->getnnz()) ? EstimateLocalFLOP<SR>(*A, *B, false, false) : 0;
  SpTuples<I, NTO>* C = nullptr;
  double t0 = MPI_Wtime();
  if (!strcmp(kernel, "hash"))        C = LocalSpGEMMHash<SR, NTO>(*A, *B, false, false, true);
  else if (!strcmp(kernel, "hash_unsorted")) C = LocalSpGEMMHash<SR, NTO>(*A, *B, false, false, false);
  else if (!strcmp(kernel, "heap"))   C = LocalSpGEMM<SR, NTO>(*A, *B, false, false);
  else if (!strcmp(kernel, "hybrid")) C = LocalHybridSpGEMM<SR, NTO>(*A, *B, false, false);
  else { fprintf(stderr, "unknown kernel %s\n", kernel); return 2; }
  double t1 = MPI_Wtime();
  long dups = count_dups<NTO>(*C);
  write_tuples<NTO>(out, *C, RA.nrow, RB.ncol);
  printf("{\"kernel\":\"%s\",\"flops\":%ld,\"nnzC\":%ld,\"dups\":%ld,\"seconds\":%.6f}\n",
         kernel, (long)flops, (long)C->getnnz(), dups, t1 - t0);
  delete C; delete A; delete B;
  return 0;
}

static int dispatch_mult(const char* sr, const char* kernel, const char* fa, const char* fb, const char* out) {
  RawCsc A = read_bin(fa), B = read_bin(fb);
  std::string s(sr);
  // Semirings.h: PlusTimesSRing 212-233, MinPlusSRing 235-255, Select2ndSRing 143-163,
  // SelectMaxSRing 165-190 and its <bool,T2> specialisation 191-210.
  if (s == "plus_times_f64") return run_mult<PlusTimesSRing<double, double>, double, double, double>(kernel, A, B, out);
  if (s == "plus_times_i64") return run_mult<PlusTimesSRing<int64_t, int64_t>, int64_t, int64_t, int64_t>(kernel, A, B, out);
  if (s == "min_plus_i64")   return run_mult<MinPlusSRing<int64_t, int64_t>, int64_t, int64_t, int64_t>(kernel, A, B, out);
  if (s == "min_plus_f64")   return run_mult<MinPlusSRing<double, double>, double, double, double>(kernel, A, B, out);
  if (s == "select2nd_i64")  return run_mult<Select2ndSRing<int64_t, int64_t, int64_t>, int64_t, int64_t, int64_t>(kernel, A, B, out);
  if (s == "select_max_i64") return run_mult<SelectMaxSRing<int64_t, int64_t>, int64_t, int64_t, int64_t>(kernel, A, B, out);
  if (s == "bool_max_i64")   return run_mult<SelectMaxSRing<bool, int64_t>, int64_t, bool, int64_t>(kernel, A, B, out);
  fprintf(stderr, "unknown semiring %s\n", sr); return 2;
}

// 1-rank distributed driver (PSpGEMM -> Mult_AnXBn_Synch); inputs read independently.
static int run_synch(const char* fa, const char* fb, const char* out) {
  typedef SpDCCols<I, double> DCC; typedef SpParMat<I, double, DCC> PM;
  RawCsc RA = read_bin(fa), RB = read_bin(fb);
  std::shared_ptr<CommGrid> g(new CommGrid(MPI_COMM_WORLD, 0, 0));
  if (g->GetSize() != 1) { fprintf(stderr, "synch probe is 1-rank only\n"); return 2; }
  DCC* a = to_dcc<double>(RA); DCC* b = to_dcc<double>(RB);
  PM A(a, g), B(b, g);
  double t0 = MPI_Wtime();
  PM C = Mult_AnXBn_Synch<PlusTimesSRing<double, double>, double, DCC>(A, B);
  double t1 = MPI_Wtime();
  write_dcc<double>(out, *C.seqptr());
  printf("{\"kernel\":\"synch\",\"nnzC\":%ld,\"seconds\":%.6f}\n", (long)C.getnnz(), t1 - t0);
  return 0;
}

// Graph500 Kronecker matrix exactly as the reference builds it for its R-MAT runs:
// GenGraph500Data(packed=true) (SEED env, default 0xDECAFBAD, RefGen21.h:306-318) then
// SpParMat(DistEdgeList) which sums duplicate edges (SpTuples.cpp:66-115).
static int run_gen(int scale, int ef, const char* out) {
  typedef SpDCCols<I, double> DCC; typedef SpParMat<I, double, DCC> PM;
  double init[4] = {.57, .19, .19, .05};
  DistEdgeList<I>* DEL = new DistEdgeList<I>();
  DEL->GenGraph500Data(init, scale, ef, true, true);
  PM A(*DEL, false); delete DEL;
  write_dcc<double>(out, *A.seqptr());
  printf("{\"gen\":%d,\"nnz\":%ld}\n", scale, (long)A.getnnz());
  return 0;
}

// Matrix Market read with the reference's own reader (symmetric expansion, duplicate
// handling by maximum<double>, as the survey/MultTest use it).
static int run_readmm(const char* mtx, const char* out) {
  typedef SpDCCols<I, double> DCC; typedef SpParMat<I, double, DCC> PM;
  std::shared_ptr<CommGrid> g(new CommGrid(MPI_COMM_WORLD, 0, 0));
  PM A(g);
  A.ParallelReadMM(std::string(mtx), true, maximum<double>());
  write_dcc<double>(out, *A.seqptr());
  printf("{\"readmm\":\"%s\",\"nnz\":%ld}\n", mtx, (long)A.getnnz());
  return 0;
}

// HipMCL prune/select/recover on a 1-rank SpParMat (ParFriends.h:185-353), in place.
static int run_mcl(const char* fa, double thr, long sel, long rec, double pct, const char* out) {
  typedef SpDCCols<I, double> DCC; typedef SpParMat<I, double, DCC> PM;
  RawCsc RA = read_bin(fa);
  std::shared_ptr<CommGrid> g(new CommGrid(MPI_COMM_WORLD, 0, 0));
  PM A(to_dcc<double>(RA), g);
  MCLPruneRecoverySelect(A, thr, (I)sel, (I)rec, pct, 1);
  write_dcc<double>(out, *A.seqptr());
  printf("{\"mcl\":1,\"nnz\":%ld}\n", (long)A.getnnz());
  return 0;
}

// HipMCL expansion A*A in `phases` column phases with prune after each (ParFriends.h:449-730).
static int run_memeff(const char* fa, int phases, double thr, long sel, long rec, double pct, const char* out) {
  typedef SpDCCols<I, double> DCC; typedef SpParMat<I, double, DCC> PM;
  typedef PlusTimesSRing<double, double> PTFF;
  RawCsc RA = read_bin(fa);
  std::shared_ptr<CommGrid> g(new CommGrid(MPI_COMM_WORLD, 0, 0));
  PM A(to_dcc<double>(RA), g), B(to_dcc<double>(RA), g);
  PM C = MemEfficientSpGEMM<PTFF, double, DCC>(A, B, phases, thr, (I)sel, (I)rec, pct, 1, 1, 0);
  write_dcc<double>(out, *C.seqptr());
  printf("{\"memeff\":%d,\"nnz\":%ld}\n", phases, (long)C.getnnz());
  return 0;
}

// k column-sorted lists merged by the reference's heap MultiwayMerge (MultiwayMerge.h:411-526) and hash
// MultiwayMergeHash (:536-684), both written out (outputs re-sorted column-major, as everywhere here).
template <class SR, class NT>
static int run_merge_t(int k, char** files, const char* out_heap, const char* out_hash) {
  std::vector<RawCsc> raw;
  for (int i = 0; i < k; ++i) raw.push_back(read_bin(files[i]));
  const I m = raw[0].nrow, n = raw[0].ncol;
  auto lists = [&]() {
    std::vector<SpTuples<I, NT>*> L;
    for (auto& R : raw) {
      SpDCCols<I, NT>* D = to_dcc<NT>(R);
      SpTuples<I, NT>* T = new SpTuples<I, NT>(*D);
      T->SortColBased();
      delete D;
      L.push_back(T);
    }
    return L;
  };
  std::vector<SpTuples<I, NT>*> l1 = lists(), l2 = lists();
  SpTuples<I, NT>* h = MultiwayMerge<SR>(l1, m, n, true);
  SpTuples<I, NT>* g = MultiwayMergeHash<SR>(l2, m, n, true, true);
  write_tuples<NT>(out_heap, *h, m, n);
  write_tuples<NT>(out_hash, *g, m, n);
  printf("{\"merge\":%d,\"nnz_heap\":%ld,\"nnz_hash\":%ld}\n", k, (long)h->getnnz(), (long)g->getnnz());
  delete h; delete g;
  return 0;
}

static int run_merge(const char* sr, int k, char** files, const char* oh, const char* og) {
  std::string s(sr);
  if (s == "select2nd_i64") return run_merge_t<Select2ndSRing<int64_t, int64_t, int64_t>, int64_t>(k, files, oh, og);
  if (s == "plus_times_i64") return run_merge_t<PlusTimesSRing<int64_t, int64_t>, int64_t>(k, files, oh, og);
  if (s == "min_plus_i64") return run_merge_t<MinPlusSRing<int64_t, int64_t>, int64_t>(k, files, oh, og);
  fprintf(stderr, "unknown semiring %s\n", sr); return 2;
}

int main(int argc, char** argv) {
  int prov; MPI_Init_thread(&argc, &argv, MPI_THREAD_SERIALIZED, &prov);
  int rc = 2;
  if (argc >= 2) {
    std::string cmd(argv[1]);
    if (cmd == "mult" && argc == 7) rc = dispatch_mult(argv[2], argv[3], argv[4], argv[5], argv[6]);
    else if (cmd == "synch" && argc == 5) rc = run_synch(argv[2], argv[3], argv[4]);
    else if (cmd == "gen" && argc == 5) rc = run_gen(atoi(argv[2]), atoi(argv[3]), argv[4]);
    else if (cmd == "readmm" && argc == 4) rc = run_readmm(argv[2], argv[3]);
    else if (cmd == "mcl" && argc == 8)
      rc = run_mcl(argv[2], atof(argv[3]), atol(argv[4]), atol(argv[5]), atof(argv[6]), argv[7]);
    else if (cmd == "merge" && argc >= 6 && argc == 6 + atoi(argv[3]))
      rc = run_merge(argv[2], atoi(argv[3]), argv + 4, argv[4 + atoi(argv[3])], argv[5 + atoi(argv[3])]);
    else if (cmd == "memeff" && argc == 9)
      rc = run_memeff(argv[2], atoi(argv[3]), atof(argv[4]), atol(argv[5]), atol(argv[6]), atof(argv[7]), argv[8]);
  }
  if (rc == 2 && argc < 3)
    fprintf(stderr, "usage: refprobe mult <sr> <hash|hash_unsorted|heap|hybrid> A.bin B.bin C.bin | synch A B C | gen scale ef out | readmm in.mtx out | mcl A thr sel rec pct out | memeff A phases thr sel rec pct out | merge <sr> k L1..Lk heap.out hash.out\n");
  MPI_Finalize();
  return rc;
}
