// oracle/ref/refbench.cpp -- TEST/BENCH INFRASTRUCTURE ONLY: times the *reference's own* CPU SpGEMM.
//
// bench.py's `cpu_baseline` leg runs this binary (built from the reference's headers and sources where they lie
// under /root/reference by oracle/ref/Makefile; the binary travels to the GPU box in oracle/_ref/) on the same
// bounded sample of the benchmarked product that the GPU result is checked on: A = the R-MAT matrix, B = every
// s-th column of A.  It times, with all the OpenMP threads OMP_NUM_THREADS gives it, at one MPI rank:
//   LocalSpGEMMHash<PlusTimesSRing<double,double>,double>(A, B, false, false, true)   mtSpGEMM.h:465-661
//   Mult_AnXBn_Synch<PlusTimesSRing<double,double>,double,SpDCCols>(A, B) on a 1x1 CommGrid
//                                                          ParFriends.h:1004-1108 (local hash + MultiwayMerge + DCSC)
// and prints one JSON line per timed call with the multiplies (EstimateLocalFLOP, mtSpGEMM.h:667-694), nnz(C)
// and an order-independent checksum of the output entries (sum over entries of mix(row, col) ^ mix(value bits),
// mod 2^64), which bench.py compares with the same checksum of the GPU product's sampled columns.
//
// usage: refbench A.bin stride_hash stride_synch      (A.bin: the CBM1 format of refprobe.cpp, values f64)
#include <mpi.h>
#include <omp.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <tuple>
#include "CombBLAS/CombBLAS.h"
using namespace combblas;

typedef int64_t I;
typedef SpDCCols<I, double> DCC;
typedef PlusTimesSRing<double, double> PTDD;

struct RawMat {
  I nrow = 0, ncol = 0, nnz = 0;
  std::vector<I> cp, ir;
  std::vector<double> val;
};

static bool read_cbm(const char* path, RawMat* M) {
  FILE* f = fopen(path, "rb");
  if (!f) { perror(path); return false; }
  char mg[4];
  int32_t vt = -1;
  bool ok = fread(mg, 1, 4, f) == 4 && !memcmp(mg, "CBM1", 4) && fread(&vt, 4, 1, f) == 1 && vt == 0 &&
            fread(&M->nrow, 8, 1, f) == 1 && fread(&M->ncol, 8, 1, f) == 1 && fread(&M->nnz, 8, 1, f) == 1;
  if (ok) {
    M->cp.resize(M->ncol + 1);
    M->ir.resize(M->nnz);
    M->val.resize(M->nnz);
    ok = fread(M->cp.data(), 8, M->ncol + 1, f) == (size_t)(M->ncol + 1) &&
         fread(M->ir.data(), 8, M->nnz, f) == (size_t)M->nnz && fread(M->val.data(), 8, M->nnz, f) == (size_t)M->nnz;
  }
  fclose(f);
  if (!ok) fprintf(stderr, "refbench: %s is not a CBM1 f64 matrix\n", path);
  return ok;
}

// columns 0, s, 2s, ... of M as a SpDCCols (column c of the result = column c*s of M)
static DCC* columns_as_dcc(const RawMat& M, I stride) {
  const I nc = (M.ncol + stride - 1) / stride;
  I nz = 0;
  for (I c = 0; c < nc; ++c) nz += M.cp[c * stride + 1] - M.cp[c * stride];
  std::tuple<I, I, double>* t = new std::tuple<I, I, double>[nz > 0 ? nz : 1];
  I p = 0;
  for (I c = 0; c < nc; ++c)
    for (I k = M.cp[c * stride]; k < M.cp[c * stride + 1]; ++k) t[p++] = std::make_tuple(M.ir[k], c, M.val[k]);
  SpTuples<I, double> T(nz, M.nrow, nc, t, true, false);   // column-sorted, rows ascending: no re-sort
  return new DCC(T, false);
}

static inline uint64_t mix64(uint64_t x) {   // splitmix64 finaliser
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}
static inline uint64_t entry_hash(I r, I c, double v) {
  uint64_t b;
  memcpy(&b, &v, 8);
  return mix64(((uint64_t)r << 32) ^ (uint64_t)c) ^ mix64(b);
}

static uint64_t checksum(SpTuples<I, double>& T) {
  uint64_t s = 0;
  for (I k = 0; k < T.getnnz(); ++k) s += entry_hash(T.rowindex(k), T.colindex(k), T.numvalue(k));
  return s;
}

static uint64_t checksum(DCC& D) {
  SpTuples<I, double> T(D);
  return checksum(T);
}

int main(int argc, char** argv) {
  int prov;
  MPI_Init_thread(&argc, &argv, MPI_THREAD_SERIALIZED, &prov);
  int rc = 2;
  RawMat M;
  if (argc == 4 && read_cbm(argv[1], &M)) {
    const I s_hash = atol(argv[2]), s_synch = atol(argv[3]);
    const int threads = omp_get_max_threads();
    DCC* A = columns_as_dcc(M, 1);
    if (s_hash > 0) {
      DCC* B = columns_as_dcc(M, s_hash);
      const I flops = EstimateLocalFLOP<PTDD>(*A, *B, false, false);
      double t0 = MPI_Wtime();
      SpTuples<I, double>* C = LocalSpGEMMHash<PTDD, double>(*A, *B, false, false, true);
      double t1 = MPI_Wtime();
      printf("{\"call\":\"LocalSpGEMMHash\",\"stride\":%ld,\"columns\":%ld,\"multiplies\":%ld,\"nnzC\":%ld,"
             "\"seconds\":%.6f,\"omp_threads\":%d,\"mpi_ranks\":1,\"checksum\":\"%016llx\"}\n",
             (long)s_hash, (long)B->getncol(), (long)flops, (long)C->getnnz(), t1 - t0, threads,
             (unsigned long long)checksum(*C));
      fflush(stdout);
      delete C;
      delete B;
    }
    if (s_synch > 0) {
      typedef SpParMat<I, double, DCC> PM;
      std::shared_ptr<CommGrid> g(new CommGrid(MPI_COMM_WORLD, 0, 0));
      DCC* B = columns_as_dcc(M, s_synch);
      const I flops = EstimateLocalFLOP<PTDD>(*A, *B, false, false);
      PM PA(new DCC(*A), g), PB(B, g);
      double t0 = MPI_Wtime();
      PM C = Mult_AnXBn_Synch<PTDD, double, DCC>(PA, PB);
      double t1 = MPI_Wtime();
      printf("{\"call\":\"Mult_AnXBn_Synch\",\"stride\":%ld,\"columns\":%ld,\"multiplies\":%ld,\"nnzC\":%ld,"
             "\"seconds\":%.6f,\"omp_threads\":%d,\"mpi_ranks\":1,\"checksum\":\"%016llx\"}\n",
             (long)s_synch, (long)C.getncol(), (long)flops, (long)C.getnnz(), t1 - t0, threads,
             (unsigned long long)checksum(*C.seqptr()));
      fflush(stdout);
    }
    delete A;
    rc = 0;
  } else if (argc != 4) {
    fprintf(stderr, "usage: refbench A.bin stride_hash stride_synch   (0 skips a call)\n");
  }
  MPI_Finalize();
  return rc;
}
