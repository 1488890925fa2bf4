// oracle/ref/refrestrict.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never measured).
//
// Runs the reference's own Galerkin restriction operator at ONE rank and writes R and R^T:
//   RestrictionOp(CCGrid&, SpDCCols*, R, RT)   3DSpGEMM/RestrictionOp.h:196-291
//   MIS2 (MIS on A u A^2)                      3DSpGEMM/RestrictionOp.h:116-193
//   FullyDistVec::RandPerm                     include/CombBLAS/FullyDistVec.cpp:783-900
// Compiled with -DDETERMINISTIC (see Makefile): the reference's own switch that seeds GlobalMT with 1
// (RestrictionOp.h:15-16) and RandPerm with 1383098845 (FullyDistVec.cpp:785-786), so at one rank the
// output is a fixed function of the input.  Matrix files use refprobe's CBM1 format.
//
// usage: refrestrict A.bin R.bin RT.bin
#include <mpi.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <tuple>
#include "CombBLAS/CombBLAS.h"
#include "3DSpGEMM/CCGrid.h"
#include "3DSpGEMM/RestrictionOp.h"
using namespace combblas;

typedef int64_t I;

static SpDCCols<I, double>* read_bin(const char* path, I* nrow, I* ncol) {
  FILE* f = fopen(path, "rb");
  if (!f) { perror(path); exit(2); }
  char mg[4];
  int32_t vt = 0;
  I nnz = 0;
  if (fread(mg, 1, 4, f) != 4 || memcmp(mg, "CBM1", 4)) { fprintf(stderr, "bad magic %s\n", path); exit(2); }
  fread(&vt, 4, 1, f); fread(nrow, 8, 1, f); fread(ncol, 8, 1, f); fread(&nnz, 8, 1, f);
  std::vector<I> cp(*ncol + 1), ir(nnz);
  fread(cp.data(), 8, *ncol + 1, f); fread(ir.data(), 8, nnz, f);
  std::vector<double> v(nnz);
  if (vt == 0) fread(v.data(), 8, nnz, f);
  else if (vt == 1) { std::vector<int64_t> w(nnz); fread(w.data(), 8, nnz, f); for (I k = 0; k < nnz; ++k) v[k] = (double)w[k]; }
  else { std::vector<uint8_t> w(nnz); fread(w.data(), 1, nnz, f); for (I k = 0; k < nnz; ++k) v[k] = w[k]; }
  fclose(f);
  std::tuple<I, I, double>* t = new std::tuple<I, I, double>[nnz > 0 ? nnz : 1];
  I p = 0;
  for (I c = 0; c < *ncol; ++c)
    for (I k = cp[c]; k < cp[c + 1]; ++k) t[p++] = std::make_tuple(ir[k], c, v[k]);
  SpTuples<I, double> T(nnz, *nrow, *ncol, t, true, false);
  return new SpDCCols<I, double>(T, false);
}

static void write_dcc(const char* path, SpDCCols<I, double>& D) {
  SpTuples<I, double> T(D);
  T.SortColBased();
  const I nrow = D.getnrow(), ncol = D.getncol(), nnz = T.getnnz();
  std::vector<I> cp(ncol + 1, 0);
  for (I k = 0; k < nnz; ++k) cp[T.colindex(k) + 1]++;
  for (I c = 0; c < ncol; ++c) cp[c + 1] += cp[c];
  FILE* f = fopen(path, "wb");
  fwrite("CBM1", 1, 4, f);
  int32_t vt = 0;
  fwrite(&vt, 4, 1, f);
  fwrite(&nrow, 8, 1, f); fwrite(&ncol, 8, 1, f); fwrite(&nnz, 8, 1, f);
  fwrite(cp.data(), 8, ncol + 1, f);
  for (I k = 0; k < nnz; ++k) { I r = T.rowindex(k); fwrite(&r, 8, 1, f); }
  for (I k = 0; k < nnz; ++k) { double x = T.numvalue(k); fwrite(&x, 8, 1, f); }
  fclose(f);
}

int main(int argc, char** argv) {
  int prov;
  MPI_Init_thread(&argc, &argv, MPI_THREAD_SERIALIZED, &prov);
  int rc = 2;
  if (argc == 4) {
    int np = 0;
    MPI_Comm_size(MPI_COMM_WORLD, &np);
    if (np != 1) {
      fprintf(stderr, "refrestrict is 1-rank only\n");
    } else {
      I nrow = 0, ncol = 0;
      SpDCCols<I, double>* A = read_bin(argv[1], &nrow, &ncol);
      CCGrid CMG(1, 1);
      SpDCCols<I, double>* R = nullptr;
      SpDCCols<I, double>* RT = nullptr;
      RestrictionOp(CMG, A, R, RT);
      write_dcc(argv[2], *R);
      write_dcc(argv[3], *RT);
      printf("{\"restrict\":1,\"n\":%ld,\"naggr\":%ld,\"nnzR\":%ld}\n", (long)R->getnrow(), (long)R->getncol(),
             (long)R->getnnz());
      delete R; delete RT; delete A;
      rc = 0;
    }
  } else {
    fprintf(stderr, "usage: refrestrict A.bin R.bin RT.bin\n");
  }
  MPI_Finalize();
  return rc;
}
