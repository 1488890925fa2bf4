/*
 * combblas_gpu.h -- C++ drop-in for the reference's local SpGEMM plugin point, over the C ABI
 * (include/cbgpu.h, libcbgpu.so).  Include it after CombBLAS/CombBLAS.h; it adds
 *
 *   combblas::gpu::LocalSpGEMMHash<SR, NTO>(A, B, clearA, clearB, sort)   mtSpGEMM.h:465-470
 *   combblas::gpu::LocalHybridSpGEMM<SR, NTO>(A, B, clearA, clearB, aux)  mtSpGEMM.h:212-217
 *   combblas::gpu::LocalSpGEMM<SR, NTO>(A, B, clearA, clearB)             mtSpGEMM.h:73-78
 *   combblas::gpu::MultiwayMerge<SR>(lists, mdim, ndim, delarrs)          MultiwayMerge.h:411-412
 *   combblas::gpu::MultiwayMergeHash<SR>(lists, mdim, ndim, delarrs, sorted) MultiwayMerge.h:536-537
 *   combblas::gpu::EstimateLocalFLOP<SR>(A, B)                             mtSpGEMM.h:667-694
 *   combblas::gpu::MCLPruneRecoverySelect(A, thr, select, recover, pct, v) ParFriends.h:185-353
 *   combblas::gpu::Mult_AnXBn_Synch<SR, NUO, UDERO>(A, B, clearA, clearB) ParFriends.h:1004-1108
 *   combblas::gpu::Mult_AnXBn_DoubleBuff / Mult_AnXBn_Overlap           ParFriends.h:798-997, 1110-1235
 *   combblas::gpu::PSpGEMM<SR>(A, B)                                      SpParMat.h:451-464
 *   combblas::gpu::Mult_AnXBn_SUMMA3D<SR, NUO, UDERO>(A3D, B3D)          ParFriends.h:2918-3208
 *   combblas::gpu::multiply(splitA, splitB, CMG, isBT, threaded)           3DSpGEMM/Multiplier.h:10-61
 *   combblas::gpu::SUMMALayer(splitA, splitB, C, CMG, isBT, threaded)      3DSpGEMM/SUMMALayer.h:24-97
 *   combblas::gpu::RestrictionOp(CMG, localmat, R, RT)                    3DSpGEMM/RestrictionOp.h:196-291
 *     (the 3DSpGEMM ones are declared when 3DSpGEMM/CCGrid.h is included before this header)
 *
 * The distributed ones run the whole SUMMA (stage broadcasts, local products, merges, fiber
 * exchange) inside libcbgpu on the device (cbg_spgemm_grid) over the SpParMat's own MPI
 * communicators (a host-staged cbg_transport built on MPI_Bcast / MPI_Alltoallv / MPI_Allgather);
 * the local block goes down once and the product comes back once (no SpTuples per stage).
 *
 * MemEfficientSpGEMM (ParFriends.h:449-730) gets the device path by calling the first and the last
 * of these in place of the reference's LocalSpGEMMHash / MCLPruneRecoverySelect.
 *
 * with the reference's signatures and conventions: A, B are SpDCCols<IT, NT> (their DCSC arrays are
 * handed to the device as they are, GetArrays order cp, jc, ir, numx); the product comes back as a
 * column-sorted SpTuples<IT, NTO>* owned by the caller; clearA / clearB delete the inputs after the
 * call (mtSpGEMM.h:644-647); an empty operand gives an empty SpTuples (mtSpGEMM.h:478-481).
 * A semiring without a device functor (anything but the six policies of Semirings.h mapped below)
 * runs the reference's own CPU template.  Device/ABI errors throw std::runtime_error; a dimension
 * mismatch throws too (the MPI drivers abort with DIMMISMATCH 3002 there).
 *
 * Not part of libcbgpu: a maintainer adds this header on the reference side.
 */
#ifndef COMBBLAS_GPU_H
#define COMBBLAS_GPU_H

#include <algorithm>
#include <cstdlib>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <tuple>
#include <type_traits>
#include <vector>

#include "cbgpu.h"

namespace combblas {
namespace gpu {

// ---------------------------------------------------------------- semiring / dtype mapping
template <class SR> struct DeviceSemiring { static constexpr bool ok = false; };
template <class T1, class T2> struct DeviceSemiring<PlusTimesSRing<T1, T2>> {
  static constexpr bool ok = true; static constexpr cbg_semiring code = CBG_SR_PLUS_TIMES; };
template <class T1, class T2> struct DeviceSemiring<MinPlusSRing<T1, T2>> {
  static constexpr bool ok = true; static constexpr cbg_semiring code = CBG_SR_MIN_PLUS; };
template <class T1, class T2, class O> struct DeviceSemiring<Select2ndSRing<T1, T2, O>> {
  static constexpr bool ok = true; static constexpr cbg_semiring code = CBG_SR_SELECT2ND; };
template <class T1, class T2> struct DeviceSemiring<SelectMaxSRing<T1, T2>> {
  static constexpr bool ok = true;
  static constexpr cbg_semiring code = std::is_same<T1, bool>::value ? CBG_SR_SELECT_MAX_BOOL : CBG_SR_SELECT_MAX; };
template <class O> struct DeviceSemiring<BoolCopy1stSRing<O>> {
  static constexpr bool ok = true; static constexpr cbg_semiring code = CBG_SR_BOOL_COPY1ST; };
template <class O> struct DeviceSemiring<BoolCopy2ndSRing<O>> {
  static constexpr bool ok = true; static constexpr cbg_semiring code = CBG_SR_BOOL_COPY2ND; };

template <class T> struct DeviceType { static constexpr bool ok = false; };
template <> struct DeviceType<double> { static constexpr bool ok = true; static constexpr cbg_dtype code = CBG_F64; };
template <> struct DeviceType<float> { static constexpr bool ok = true; static constexpr cbg_dtype code = CBG_F32; };
template <> struct DeviceType<int64_t> { static constexpr bool ok = true; static constexpr cbg_dtype code = CBG_I64; };
template <> struct DeviceType<int32_t> { static constexpr bool ok = true; static constexpr cbg_dtype code = CBG_I32; };
template <> struct DeviceType<bool> { static constexpr bool ok = true; static constexpr cbg_dtype code = CBG_BOOL; };

// host staging element of a value type (std::vector<bool> has no data(): bools travel as bytes)
template <class T> using Store = typename std::conditional<std::is_same<T, bool>::value, uint8_t, T>::type;

inline void check(cbg_status s, const char* where) {
  if (s != CBG_OK) throw std::runtime_error(std::string(where) + ": " + cbg_strerror(s));
}

// One context per process/host thread.  context(d) selects device d; without a choice, an MPI process takes its
// node-local rank's device modulo the visible devices (one GPU per rank on an 8-GPU node), any other process
// device 0.  The context may be created by one rank alone (e.g. RestrictionOp's layer rank 0), so the local rank
// comes from the launcher's environment (MPICH MPI_LOCALRANKID, Open MPI OMPI_COMM_WORLD_LOCAL_RANK, Slurm
// SLURM_LOCALID), else from the world rank -- never from a collective.
inline int node_local_device() {
  int32_t n = 0;
  if (cbg_device_count(&n) != CBG_OK || n <= 0) return 0;
  for (const char* v : {"MPI_LOCALRANKID", "OMPI_COMM_WORLD_LOCAL_RANK", "SLURM_LOCALID"})
    if (const char* x = std::getenv(v)) return std::atoi(x) % n;
  int init = 0, fin = 0, r = 0;
  MPI_Initialized(&init);
  MPI_Finalized(&fin);
  if (init && !fin) MPI_Comm_rank(MPI_COMM_WORLD, &r);
  return r % n;
}

inline cbg_ctx* context(int device = -1) {
  static thread_local cbg_ctx* ctx = nullptr;
  static thread_local int dev = 0;
  if (device >= 0 && ctx && device != dev) { cbg_destroy(ctx); ctx = nullptr; }
  if (!ctx) {
    // the library writes structs this header allocates (cbg_profile, cbg_grid_stats): refuse another ABI version
    if (cbg_abi_version() != CBG_ABI_VERSION)
      throw std::runtime_error("cbg_abi_version: libcbgpu.so is ABI " + std::to_string(cbg_abi_version()) +
                               ", this header is ABI " + std::to_string(CBG_ABI_VERSION));
    dev = device >= 0 ? device : node_local_device();
    check(cbg_init(dev, &ctx), "cbg_init");
  }
  return ctx;
}

// borrowed view of an SpDCCols (the DCSC arrays as GetArrays hands them out, SpDCCols.cpp:817-839)
template <class IT, class NT>
cbg_dcsc_view view_of(const SpDCCols<IT, NT>& M) {
  static_assert(sizeof(IT) == 4 || sizeof(IT) == 8, "IT must be a 32- or 64-bit integer");
  cbg_dcsc_view v{};
  v.nrow = M.getnrow(); v.ncol = M.getncol(); v.nnz = M.getnnz(); v.nzc = M.getnzc();
  Arr<IT, NT> arr = M.GetArrays();
  v.cp = arr.indarrs[0].addr; v.jc = arr.indarrs[1].addr; v.ir = arr.indarrs[2].addr;
  if (v.jc == nullptr) v.nzc = 0;              // empty matrix: no DCSC arrays at all
  v.idx_bytes = (int32_t)sizeof(IT); v.ptr_bytes = (int32_t)sizeof(IT);
  v.val = arr.numarrs[0].addr; v.val_type = DeviceType<NT>::code; v.on_device = 0;
  return v;
}

// device CSC result -> column-sorted SpTuples (new[] tuples, isOpNew = false)
template <class IT, class NTO>
SpTuples<IT, NTO>* to_tuples(cbg_ctx* ctx, cbg_csc_result& C) {
  std::vector<int64_t> cp(C.ncol + 1);
  std::vector<int32_t> row(C.nnz > 0 ? C.nnz : 1);
  std::vector<Store<NTO>> val(C.nnz > 0 ? C.nnz : 1);
  const int64_t nrow = C.nrow, ncol = C.ncol;
  cbg_status s = cbg_result_to_host(ctx, &C, cp.data(), row.data(), C.val ? (void*)val.data() : nullptr);
  cbg_result_free(ctx, &C);   // clears C
  check(s, "cbg_result_to_host");
  const int64_t nnz = cp[ncol];
  std::tuple<IT, IT, NTO>* t = new std::tuple<IT, IT, NTO>[nnz > 0 ? nnz : 1];
  for (int64_t j = 0; j < ncol; ++j)
    for (int64_t p = cp[j]; p < cp[j + 1]; ++p) t[p] = std::make_tuple((IT)row[p], (IT)j, (NTO)val[p]);
  return new SpTuples<IT, NTO>(nnz, (IT)nrow, (IT)ncol, t, /*sorted=*/true, /*isOpNew=*/false);
}

// ------------------------------------------------------------------------- entry points
template <class SR, class NTO, class IT, class NT1, class NT2>
SpTuples<IT, NTO>* LocalSpGEMMHash(const SpDCCols<IT, NT1>& A, const SpDCCols<IT, NT2>& B, bool clearA,
                                   bool clearB, bool sort = true) {
  // the device computes in NTO: operands must carry NTO values, or be bool patterns
  constexpr bool dev = DeviceSemiring<SR>::ok && DeviceType<NTO>::ok &&
                       (std::is_same<NT1, NTO>::value || std::is_same<NT1, bool>::value) &&
                       (std::is_same<NT2, NTO>::value || std::is_same<NT2, bool>::value);
  if constexpr (!dev) {
    return combblas::LocalSpGEMMHash<SR, NTO>(A, B, clearA, clearB, sort);   // no device functor
  } else {
    if (A.getncol() != B.getnrow()) throw std::runtime_error("LocalSpGEMMHash: DIMMISMATCH (3002)");
    cbg_ctx* ctx = context();
    cbg_dcsc_view va = view_of(A), vb = view_of(B);
    cbg_csc_result C{};
    int64_t mults = 0;
    check(cbg_spgemm_local(ctx, &va, &vb, DeviceSemiring<SR>::code, DeviceType<NTO>::code,
                           sort ? CBG_SORTED_COLS : 0u, &C, &mults), "cbg_spgemm_local");
    SpTuples<IT, NTO>* out = to_tuples<IT, NTO>(ctx, C);
    if (clearA) delete const_cast<SpDCCols<IT, NT1>*>(&A);
    if (clearB) delete const_cast<SpDCCols<IT, NT2>*>(&B);
    return out;
  }
}

template <class SR, class NTO, class IT, class NT1, class NT2>
SpTuples<IT, NTO>* LocalHybridSpGEMM(const SpDCCols<IT, NT1>& A, const SpDCCols<IT, NT2>& B, bool clearA,
                                     bool clearB, IT* aux = nullptr) {
  (void)aux;   // heap/hash switch is a CPU heuristic; the device product is always sorted
  return LocalSpGEMMHash<SR, NTO>(A, B, clearA, clearB, true);
}

template <class SR, class NTO, class IT, class NT1, class NT2>
SpTuples<IT, NTO>* LocalSpGEMM(const SpDCCols<IT, NT1>& A, const SpDCCols<IT, NT2>& B, bool clearA, bool clearB) {
  return LocalSpGEMMHash<SR, NTO>(A, B, clearA, clearB, true);
}

template <class SR, class IT, class NT1, class NT2>
int64_t EstimateLocalFLOP(const SpDCCols<IT, NT1>& A, const SpDCCols<IT, NT2>& B) {
  cbg_dcsc_view va = view_of(A), vb = view_of(B);
  int64_t mults = 0, nnzc = 0;
  check(cbg_estimate(context(), &va, &vb, &mults, &nnzc), "cbg_estimate");
  return mults;
}

// device merge of SpTuples lists of one shape (cbg_merge): duplicates combine with SR::add in list order
// (MultiwayMerge.h:357); `sorted` = whether the output's rows are sorted per column (always true here)
template <class SR, class IT, class NT>
SpTuples<IT, NT>* merge_lists(std::vector<SpTuples<IT, NT>*>& lists, IT mdim, IT ndim, bool delarrs, const char* who) {
  if (lists.empty()) return new SpTuples<IT, NT>(0, mdim, ndim);
  cbg_ctx* ctx = context();
  std::vector<cbg_csc_result> parts(lists.size());
  std::vector<std::vector<int64_t>> cps(lists.size());
  std::vector<std::vector<int32_t>> rows(lists.size());
  std::vector<std::vector<Store<NT>>> vals(lists.size());
  for (size_t l = 0; l < lists.size(); ++l) {   // SpTuples -> host CSC (column order kept) -> device (cbg_upload)
    SpTuples<IT, NT>& T = *lists[l];
    const IT m = T.getnrow(), n = T.getncol();
    if ((mdim && m != mdim) || (ndim && n != ndim)) throw std::runtime_error(std::string(who) + ": dimension mismatch");
    T.SortColBased();
    cps[l].assign(n + 1, 0);
    rows[l].resize(T.getnnz() > 0 ? T.getnnz() : 1);
    vals[l].resize(T.getnnz() > 0 ? T.getnnz() : 1);
    for (int64_t k = 0; k < T.getnnz(); ++k) {
      ++cps[l][T.colindex(k) + 1];
      rows[l][k] = (int32_t)T.rowindex(k);
      vals[l][k] = (Store<NT>)T.numvalue(k);
    }
    for (IT j = 0; j < n; ++j) cps[l][j + 1] += cps[l][j];
    cbg_dcsc_view v{};
    v.nrow = m; v.ncol = n; v.nnz = T.getnnz(); v.nzc = n;
    v.cp = cps[l].data(); v.ir = rows[l].data(); v.idx_bytes = 4; v.ptr_bytes = 8;
    v.val = vals[l].data(); v.val_type = DeviceType<NT>::code; v.on_device = 0;
    cbg_status s = cbg_upload(ctx, &v, &parts[l]);
    if (s != CBG_OK) {
      for (size_t k = 0; k < l; ++k) cbg_result_free(ctx, &parts[k]);
      check(s, "cbg_upload");
    }
  }
  cbg_csc_result C{};
  cbg_status s = cbg_merge(ctx, parts.data(), (int32_t)parts.size(), DeviceSemiring<SR>::code, DeviceType<NT>::code,
                           CBG_SORTED_COLS, &C);
  for (auto& p : parts) cbg_result_free(ctx, &p);
  check(s, "cbg_merge");
  if (delarrs)
    for (auto* T : lists) delete T;
  return to_tuples<IT, NT>(ctx, C);
}

// MultiwayMerge: column-sorted partial products of one shape -> one SpTuples (duplicates: SR::add)
template <class SR, class IT, class NT>
SpTuples<IT, NT>* MultiwayMerge(std::vector<SpTuples<IT, NT>*>& lists, IT mdim = 0, IT ndim = 0,
                                bool delarrs = false) {
  if constexpr (!(DeviceSemiring<SR>::ok && DeviceType<NT>::ok)) return combblas::MultiwayMerge<SR>(lists, mdim, ndim, delarrs);
  else return merge_lists<SR>(lists, mdim, ndim, delarrs, "MultiwayMerge");
}

// MultiwayMergeHash (MultiwayMerge.h:536-684): inputs need not be row-sorted; duplicates combine in list
// order (SR::add(curval, existing), :357).  The device merge always emits row-sorted columns, which
// is what sorted = true asks for and a valid order for sorted = false.
template <class SR, class IT, class NT>
SpTuples<IT, NT>* MultiwayMergeHash(std::vector<SpTuples<IT, NT>*>& lists, IT mdim = 0, IT ndim = 0,
                                    bool delarrs = false, bool sorted = true) {
  if constexpr (!(DeviceSemiring<SR>::ok && DeviceType<NT>::ok)) {
    return combblas::MultiwayMergeHash<SR>(lists, mdim, ndim, delarrs, sorted);
  } else {
    (void)sorted;
    return merge_lists<SR>(lists, mdim, ndim, delarrs, "MultiwayMergeHash");
  }
}

// MCLPruneRecoverySelect (ParFriends.h:185-353) on the device: the statistics, the k-th-value selection and the
// prune of every column (cbg_mcl_prune) need complete columns.  On a q x q grid each processor column's q row blocks
// are gathered column group by column group (group m of the local columns goes to the column's rank m, one
// MPI_Alltoallv; the role of the processor-column Reduce / Kselect1 exchanges, SpParMat.cpp:1413-1700), pruned on
// the device, and scattered back by row block.  A non-float NT runs the reference's own version.
template <class LIT, class NT, class DER>
void block_to_csc(DER& L, std::vector<int64_t>& cp, std::vector<int32_t>& row, std::vector<NT>& val) {
  SpTuples<LIT, NT> T(L);
  T.SortColBased();
  const int64_t ncol = L.getncol(), nnz = T.getnnz();
  cp.assign(ncol + 1, 0);
  row.resize(nnz);
  val.resize(nnz);
  for (int64_t k = 0; k < nnz; ++k) {
    ++cp[T.colindex(k) + 1];
    row[k] = (int32_t)T.rowindex(k);
    val[k] = T.numvalue(k);
  }
  for (int64_t j = 0; j < ncol; ++j) cp[j + 1] += cp[j];
}

template <class NT>
void mcl_prune_host_csc(int64_t nrow, int64_t ncol, std::vector<int64_t>& cp, std::vector<int32_t>& row,
                        std::vector<NT>& val, NT thr, int64_t sel, int64_t rec, NT pct) {
  cbg_ctx* ctx = context();
  cbg_dcsc_view v{};
  v.nrow = nrow; v.ncol = ncol; v.nnz = cp[ncol]; v.nzc = ncol;
  v.cp = cp.data(); v.ir = row.empty() ? nullptr : row.data(); v.idx_bytes = 4; v.ptr_bytes = 8;
  v.val = val.empty() ? nullptr : val.data(); v.val_type = DeviceType<NT>::code; v.on_device = 0;
  cbg_csc_result D{}, P{};
  check(cbg_upload(ctx, &v, &D), "cbg_upload");
  cbg_status s = cbg_mcl_prune(ctx, &D, (double)thr, sel, rec, (double)pct, &P, nullptr);
  cbg_result_free(ctx, &D);
  check(s, "cbg_mcl_prune");
  cp.assign(ncol + 1, 0);
  row.resize(P.nnz);
  val.resize(P.nnz);
  s = cbg_result_to_host(ctx, &P, cp.data(), P.nnz ? row.data() : nullptr, P.nnz ? val.data() : nullptr);
  cbg_result_free(ctx, &P);
  check(s, "cbg_result_to_host");
}

inline void mpi_counts(const std::vector<int64_t>& n, std::vector<int>& c, std::vector<int>& d, size_t elem) {
  c.resize(n.size());
  d.resize(n.size());
  int64_t o = 0;
  for (size_t m = 0; m < n.size(); ++m) {
    if (n[m] * (int64_t)elem > INT32_MAX || o * (int64_t)elem > INT32_MAX)
      throw std::runtime_error("MCLPruneRecoverySelect: a column exchange above 2^31 bytes per rank");
    c[m] = (int)(n[m] * (int64_t)elem);
    d[m] = (int)(o * (int64_t)elem);
    o += n[m];
  }
}

template <class IT, class NT, class DER>
void MCLPruneRecoverySelect(SpParMat<IT, NT, DER>& A, NT hardThreshold, IT selectNum, IT recoverNum,
                            NT recoverPct, int kselectVersion) {
  constexpr bool dev = std::is_same<NT, double>::value || std::is_same<NT, float>::value;
  (void)kselectVersion;   // Kselect1 / Kselect2 pick the same k-th value
  if constexpr (!dev) {
    combblas::MCLPruneRecoverySelect(A, hardThreshold, selectNum, recoverNum, recoverPct, kselectVersion);
  } else {
    typedef typename DER::LocalIT LIT;
    DER& L = A.seq();
    std::vector<int64_t> cp;
    std::vector<int32_t> row;
    std::vector<NT> val;
    block_to_csc<LIT, NT>(L, cp, row, val);
    const int64_t nrl = L.getnrow(), ncl = L.getncol();
    MPI_Comm colw = A.getcommgrid()->GetColWorld();
    int q = 1, me = 0;
    MPI_Comm_size(colw, &q);
    MPI_Comm_rank(colw, &me);
    if (q == 1) {
      mcl_prune_host_csc<NT>(nrl, ncl, cp, row, val, hardThreshold, (int64_t)selectNum, (int64_t)recoverNum, recoverPct);
    } else {
      // row offsets of the processor column's q row blocks; column groups of the local columns
      std::vector<int64_t> nrows(q), roff(q + 1, 0);
      MPI_Allgather(&nrl, 1, MPI_INT64_T, nrows.data(), 1, MPI_INT64_T, colw);
      for (int i = 0; i < q; ++i) roff[i + 1] = roff[i] + nrows[i];
      // the gather below uses MPI int counts and int32 global rows: every rank checks its own sizes and the whole
      // grid agrees (a different choice in two processor columns would mismatch the reference's row-world
      // collectives); too large anywhere -> every rank takes the reference's own prune
      {
        int64_t rtot_bound = 0;   // received entries <= the processor column's entries of my column groups
        MPI_Allreduce(&cp[ncl], &rtot_bound, 1, MPI_INT64_T, MPI_SUM, colw);
        const int64_t lim = INT32_MAX;
        int fits = roff[q] < lim && 8 * (ncl + 1) <= lim && 8 * (int64_t)q * (ncl / q + ncl % q + 1) <= lim &&
                   (int64_t)std::max(sizeof(NT), (size_t)4) * rtot_bound <= lim;
        int all = 0;
        MPI_Allreduce(&fits, &all, 1, MPI_INT, MPI_MIN, A.getcommgrid()->GetWorld());
        if (!all) {
          combblas::MCLPruneRecoverySelect(A, hardThreshold, selectNum, recoverNum, recoverPct, kselectVersion);
          return;
        }
      }
      auto grp = [&](int m, int64_t n, int64_t* g0, int64_t* g1) {
        *g0 = (n / q) * m;
        *g1 = m == q - 1 ? n : *g0 + n / q;
      };
      // 1. gather: group m of my columns (counts, rows, values) -> rank m of the processor column
      std::vector<int64_t> scol(q), snz(q), rcol(q), rnz(q);
      for (int m = 0; m < q; ++m) {
        int64_t g0, g1;
        grp(m, ncl, &g0, &g1);
        scol[m] = g1 - g0;
        snz[m] = cp[g1] - cp[g0];
      }
      MPI_Alltoall(snz.data(), 1, MPI_INT64_T, rnz.data(), 1, MPI_INT64_T, colw);
      MPI_Alltoall(scol.data(), 1, MPI_INT64_T, rcol.data(), 1, MPI_INT64_T, colw);
      const int64_t ng = rcol[0];   // every source holds the same local columns (one processor column)
      std::vector<int64_t> scnt(ncl), rcnt((size_t)q * ng);
      for (int64_t j = 0; j < ncl; ++j) scnt[j] = cp[j + 1] - cp[j];
      int64_t rtot = 0;
      for (int i = 0; i < q; ++i) rtot += rnz[i];
      std::vector<int32_t> rrow(rtot);
      std::vector<NT> rval(rtot);
      std::vector<int> sc, sd, rc, rd;
      mpi_counts(scol, sc, sd, 8); mpi_counts(rcol, rc, rd, 8);
      MPI_Alltoallv(scnt.data(), sc.data(), sd.data(), MPI_BYTE, rcnt.data(), rc.data(), rd.data(), MPI_BYTE, colw);
      mpi_counts(snz, sc, sd, 4); mpi_counts(rnz, rc, rd, 4);
      MPI_Alltoallv(row.data(), sc.data(), sd.data(), MPI_BYTE, rrow.data(), rc.data(), rd.data(), MPI_BYTE, colw);
      mpi_counts(snz, sc, sd, sizeof(NT)); mpi_counts(rnz, rc, rd, sizeof(NT));
      MPI_Alltoallv(val.data(), sc.data(), sd.data(), MPI_BYTE, rval.data(), rc.data(), rd.data(), MPI_BYTE, colw);
      // complete columns: for every column, source 0's rows (+ roff[0]), then source 1's, ...
      std::vector<int64_t> fcp(ng + 1, 0);
      for (int i = 0; i < q; ++i)
        for (int64_t c = 0; c < ng; ++c) fcp[c + 1] += rcnt[(size_t)i * ng + c];
      for (int64_t c = 0; c < ng; ++c) fcp[c + 1] += fcp[c];
      std::vector<int32_t> frow(rtot);
      std::vector<NT> fval(rtot);
      {
        std::vector<int64_t> cur(fcp.begin(), fcp.end() - 1);
        int64_t src = 0;
        for (int i = 0; i < q; ++i)
          for (int64_t c = 0; c < ng; ++c)
            for (int64_t k = 0; k < rcnt[(size_t)i * ng + c]; ++k, ++src) {
              frow[cur[c]] = (int32_t)(rrow[src] + roff[i]);
              fval[cur[c]++] = rval[src];
            }
      }
      // 2. prune the complete columns on the device
      mcl_prune_host_csc<NT>(roff[q], ng, fcp, frow, fval, hardThreshold, (int64_t)selectNum, (int64_t)recoverNum,
                             recoverPct);
      // 3. scatter: row block i of the pruned group -> rank i (counts per column, rows rebased, values)
      std::vector<int64_t> bcnt((size_t)q * ng, 0), bnz(q, 0), bcol(q, ng);
      for (int64_t c = 0; c < ng; ++c)
        for (int64_t k = fcp[c]; k < fcp[c + 1]; ++k) {
          const int i = (int)(std::upper_bound(roff.begin(), roff.end(), (int64_t)frow[k]) - roff.begin()) - 1;
          ++bcnt[(size_t)i * ng + c];
          ++bnz[i];
        }
      std::vector<int32_t> brow(fcp[ng]);
      std::vector<NT> bval(fcp[ng]);
      {
        std::vector<int64_t> boff(q + 1, 0);
        for (int i = 0; i < q; ++i) boff[i + 1] = boff[i] + bnz[i];
        for (int64_t c = 0; c < ng; ++c)   // rows ascend within a column, so each block's entries stay in order
          for (int64_t k = fcp[c]; k < fcp[c + 1]; ++k) {
            const int i = (int)(std::upper_bound(roff.begin(), roff.end(), (int64_t)frow[k]) - roff.begin()) - 1;
            brow[boff[i]] = (int32_t)(frow[k] - roff[i]);
            bval[boff[i]++] = fval[k];
          }
      }
      std::vector<int64_t> gnz(q), gcol(q);
      MPI_Alltoall(bnz.data(), 1, MPI_INT64_T, gnz.data(), 1, MPI_INT64_T, colw);
      MPI_Alltoall(bcol.data(), 1, MPI_INT64_T, gcol.data(), 1, MPI_INT64_T, colw);
      std::vector<int64_t> gcnt(ncl);
      int64_t gtot = 0;
      for (int m = 0; m < q; ++m) gtot += gnz[m];
      row.resize(gtot);
      val.resize(gtot);
      mpi_counts(bcol, sc, sd, 8); mpi_counts(gcol, rc, rd, 8);
      MPI_Alltoallv(bcnt.data(), sc.data(), sd.data(), MPI_BYTE, gcnt.data(), rc.data(), rd.data(), MPI_BYTE, colw);
      mpi_counts(bnz, sc, sd, 4); mpi_counts(gnz, rc, rd, 4);
      MPI_Alltoallv(brow.data(), sc.data(), sd.data(), MPI_BYTE, row.data(), rc.data(), rd.data(), MPI_BYTE, colw);
      mpi_counts(bnz, sc, sd, sizeof(NT)); mpi_counts(gnz, rc, rd, sizeof(NT));
      MPI_Alltoallv(bval.data(), sc.data(), sd.data(), MPI_BYTE, val.data(), rc.data(), rd.data(), MPI_BYTE, colw);
      // the q groups arrive in column order: the local block's columns, concatenated
      cp.assign(ncl + 1, 0);
      for (int64_t j = 0; j < ncl; ++j) cp[j + 1] = cp[j] + gcnt[j];
    }
    // host CSC -> the local block (column-sorted tuples, rows ascending)
    const int64_t nnz = cp[ncl];
    std::tuple<LIT, LIT, NT>* t = new std::tuple<LIT, LIT, NT>[nnz > 0 ? nnz : 1];
    for (int64_t j = 0; j < ncl; ++j)
      for (int64_t k = cp[j]; k < cp[j + 1]; ++k) t[k] = std::make_tuple((LIT)row[k], (LIT)j, val[k]);
    SpTuples<LIT, NT> T(nnz, (LIT)nrl, (LIT)ncl, t, true, false);
    L = DER(T, false);
  }
}

// --------------------------------------------------------------------- distributed drivers
// MPI transport for cbg_grid: host buffers (host_buffers = 1), the grid's four communicators.
struct MpiTransport {
  MPI_Comm comm[4];   // CBG_GROUP_ROW, COL, FIBER, WORLD
  static constexpr int64_t kChunk = 1 << 30;
  static int32_t bcast(void* u, int32_t g, void* buf, int64_t bytes, int32_t root) {
    MPI_Comm c = ((MpiTransport*)u)->comm[g];
    for (int64_t o = 0; o < bytes; o += kChunk) {
      const int n = (int)std::min<int64_t>(kChunk, bytes - o);
      if (MPI_Bcast((char*)buf + o, n, MPI_BYTE, root, c) != MPI_SUCCESS) return 1;
    }
    return 0;
  }
  static int32_t alltoallv(void* u, int32_t g, const void* send, const int64_t* sb, void* recv, const int64_t* rb) {
    MPI_Comm c = ((MpiTransport*)u)->comm[g];
    int P = 0;
    MPI_Comm_size(c, &P);
    std::vector<int> sc(P), rc(P), sd(P), rd(P);
    int64_t so = 0, ro = 0;
    for (int m = 0; m < P; ++m) {
      if (sb[m] > INT32_MAX || rb[m] > INT32_MAX || so > INT32_MAX || ro > INT32_MAX) return 2;   // MPI int counts
      sc[m] = (int)sb[m]; rc[m] = (int)rb[m]; sd[m] = (int)so; rd[m] = (int)ro;
      so += sb[m]; ro += rb[m];
    }
    return MPI_Alltoallv(send, sc.data(), sd.data(), MPI_BYTE, recv, rc.data(), rd.data(), MPI_BYTE, c) == MPI_SUCCESS ? 0 : 1;
  }
  static int32_t allgather(void* u, int32_t g, const void* send, void* recv, int64_t bytes) {
    MPI_Comm c = ((MpiTransport*)u)->comm[g];
    return MPI_Allgather(send, (int)bytes, MPI_BYTE, recv, (int)bytes, MPI_BYTE, c) == MPI_SUCCESS ? 0 : 1;
  }
};

struct GridHandle {
  MpiTransport mt;
  cbg_grid* grid = nullptr;
  ~GridHandle() { if (grid) cbg_grid_destroy(grid); }
};

// The grid under the distributed drivers: the library's own RCCL communicators (ncclCommInitRank on the world +
// ncclCommSplit into row / column / fiber; device buffers, broadcasts and the fiber exchange on a communication
// stream, over xGMI between the node's GPUs), the unique id handed out by an MPI_Bcast from world rank 0.
// CBG_GRID_TRANSPORT=mpi takes the host-staged MPI transport instead (MpiTransport: D2H, MPI, H2D).
// grid_rank: the rank's position l*rows*cols + i*cols + j in the library's grid numbering (default: its
// rank in `world`, which is that numbering for CommGrid / CommGrid3D; CCGrid numbers layers fastest)
// what the last distributed driver's grid ran over (cbg_grid_query: rccl = 1 and the members RCCL counts per
// communicator, or the caller transport's group sizes)
inline cbg_grid_info& last_grid_info() {
  static thread_local cbg_grid_info gi{};
  return gi;
}

inline bool grid_over_mpi() {
  const char* t = std::getenv("CBG_GRID_TRANSPORT");
  return t && std::string(t) == "mpi";
}

inline cbg_grid* make_grid(GridHandle& h, MPI_Comm world, MPI_Comm row, MPI_Comm col, MPI_Comm fiber, int layers,
                           int rows, int cols, int grid_rank = -1) {
  int wsize = 0, wrank = 0;
  MPI_Comm_size(world, &wsize);
  MPI_Comm_rank(world, &wrank);
  const int grank = grid_rank >= 0 ? grid_rank : wrank;
  if (!grid_over_mpi()) {
    // every rank learns whether rank 0 got an id, then every rank whether all communicators came up: a failure
    // takes every rank to the MPI transport together instead of leaving some blocked in a collective (e.g. ranks
    // sharing one GPU, which RCCL refuses without NCCL_HOSTID)
    char id[128] = {0};
    int ok = wrank == 0 ? (cbg_rccl_unique_id(id) == CBG_OK) : 1;
    MPI_Bcast(&ok, 1, MPI_INT, 0, world);
    cbg_status s = CBG_ECOMM;
    if (ok) {
      MPI_Bcast(id, 128, MPI_BYTE, 0, world);
      s = cbg_grid_create_rccl(context(), id, wsize, grank, layers, rows, cols, &h.grid);
    }
    int mine = ok && s == CBG_OK, all = 0;
    MPI_Allreduce(&mine, &all, 1, MPI_INT, MPI_MIN, world);
    if (all) {
      check(cbg_grid_query(h.grid, &last_grid_info()), "cbg_grid_query");
      return h.grid;
    }
    if (h.grid) { cbg_grid_destroy(h.grid); h.grid = nullptr; }
    static bool warned = false;
    if (!warned && wrank == 0)
      fprintf(stderr, "combblas_gpu: RCCL grid setup failed (%s); using the MPI transport\n",
              cbg_strerror(s == CBG_OK ? CBG_ECOMM : s));
    warned = true;
  }
  h.mt.comm[CBG_GROUP_ROW] = row; h.mt.comm[CBG_GROUP_COL] = col;
  h.mt.comm[CBG_GROUP_FIBER] = fiber; h.mt.comm[CBG_GROUP_WORLD] = world;
  cbg_transport t{};
  t.user = &h.mt; t.bcast = &MpiTransport::bcast; t.alltoallv = &MpiTransport::alltoallv;
  t.allgather = &MpiTransport::allgather; t.host_buffers = 1;
  check(cbg_grid_create(context(), &t, wsize, grank, layers, rows, cols, &h.grid), "cbg_grid_create");
  check(cbg_grid_query(h.grid, &last_grid_info()), "cbg_grid_query");
  return h.grid;
}

// Grids are cached on the grid's row communicator (an MPI attribute; its delete callback destroys the grids when
// the CommGrid / CCGrid that owns the communicator frees it), keyed by the other communicators, the shape and the
// transport: a driver called once per iteration (HipMCL's MemEfficientSpGEMM loop, MCL.cpp:573-587) sets up its
// RCCL communicators once.  grid_creations() counts the setups of this process.
struct GridCacheEntry {
  MPI_Comm world, col, fiber;
  int layers, rows, cols, grank;
  bool mpi;
  std::unique_ptr<GridHandle> h;
};
struct GridCache {
  std::vector<GridCacheEntry> v;
};
// every live cache: the reference's CommGrid/CCGrid often never free their communicators (CCGrid.h keeps rowWorld),
// and MPI_Finalize runs delete callbacks only on MPI_COMM_SELF -- so a COMM_SELF attribute (set with the first cache)
// destroys whatever grids are still cached when MPI finalizes
inline std::vector<GridCache*>& live_grid_caches() {
  static std::vector<GridCache*> v;
  return v;
}
inline int grid_cache_delete(MPI_Comm, int, void* attr, void*) {
  auto& live = live_grid_caches();
  live.erase(std::remove(live.begin(), live.end(), (GridCache*)attr), live.end());
  delete (GridCache*)attr;
  return MPI_SUCCESS;
}
inline int grid_caches_finalize(MPI_Comm, int, void*, void*) {
  auto& live = live_grid_caches();
  for (GridCache* gc : live) gc->v.clear();   // the grids go; the (emptied) caches stay with their communicators
  return MPI_SUCCESS;
}
inline int grid_cache_keyval() {
  static int kv = MPI_KEYVAL_INVALID;
  if (kv == MPI_KEYVAL_INVALID) {
    MPI_Comm_create_keyval(MPI_COMM_NULL_COPY_FN, &grid_cache_delete, &kv, nullptr);
    int fkv = MPI_KEYVAL_INVALID;
    MPI_Comm_create_keyval(MPI_COMM_NULL_COPY_FN, &grid_caches_finalize, &fkv, nullptr);
    MPI_Comm_set_attr(MPI_COMM_SELF, fkv, nullptr);
  }
  return kv;
}
inline int& grid_creations() {
  static int n = 0;
  return n;
}
inline cbg_grid* cached_grid(MPI_Comm world, MPI_Comm row, MPI_Comm col, MPI_Comm fiber, int layers, int rows, int cols,
                             int grid_rank = -1) {
  const int kv = grid_cache_keyval();
  GridCache* gc = nullptr;
  int flag = 0;
  MPI_Comm_get_attr(row, kv, &gc, &flag);
  if (!flag || !gc) {
    gc = new GridCache;
    MPI_Comm_set_attr(row, kv, gc);
    live_grid_caches().push_back(gc);
  }
  const bool mpi = grid_over_mpi();
  for (GridCacheEntry& e : gc->v)
    if (e.world == world && e.col == col && e.fiber == fiber && e.layers == layers && e.rows == rows &&
        e.cols == cols && e.grank == grid_rank && e.mpi == mpi) {
      check(cbg_grid_query(e.h->grid, &last_grid_info()), "cbg_grid_query");
      return e.h->grid;
    }
  std::unique_ptr<GridHandle> h(new GridHandle);
  make_grid(*h, world, row, col, fiber, layers, rows, cols, grid_rank);
  ++grid_creations();
  gc->v.push_back(GridCacheEntry{world, col, fiber, layers, rows, cols, grid_rank, mpi, std::move(h)});
  return gc->v.back().h->grid;
}


// the rank's product piece (device CSC) -> UDERO via column-sorted SpTuples
template <class IU, class NUO, class UDERO>
UDERO* to_local(cbg_csc_result& C) {
  typedef typename UDERO::LocalIT LIT;
  SpTuples<LIT, NUO>* t = to_tuples<LIT, NUO>(context(), C);
  UDERO* D = new UDERO(*t, false);
  delete t;
  return D;
}

template <class SR, class NUO, class UDERO, class IU, class NU1, class NU2, class UDERA, class UDERB>
SpParMat<IU, NUO, UDERO> summa2d(SpParMat<IU, NU1, UDERA>& A, SpParMat<IU, NU2, UDERB>& B, bool clearA, bool clearB,
                                 uint32_t flags) {
  std::shared_ptr<CommGrid> GA = A.getcommgrid(), GB = B.getcommgrid();
  if (A.getncol() != B.getnrow() || !(*GA == *GB)) throw std::runtime_error("Mult_AnXBn: DIMMISMATCH (3002)");
  cbg_grid* grid = cached_grid(GA->GetWorld(), GA->GetRowWorld(), GA->GetColWorld(), MPI_COMM_SELF, 1,
                               GA->GetGridRows(), GA->GetGridCols());
  cbg_dcsc_view va = view_of(*A.seqptr()), vb = view_of(*B.seqptr());
  cbg_csc_result C{};
  cbg_grid_stats st{};
  check(cbg_spgemm_grid(grid, &va, &vb, DeviceSemiring<SR>::code, DeviceType<NUO>::code,
                        CBG_SORTED_COLS | flags, &C, &st), "cbg_spgemm_grid");
  UDERO* D = to_local<IU, NUO, UDERO>(C);
  if (clearA) A.FreeMemory();
  if (clearB) B.FreeMemory();
  return SpParMat<IU, NUO, UDERO>(D, GA);
}

template <class SR, class NUO, class UDERO, class IU, class NU1, class NU2, class UDERA, class UDERB>
SpParMat<IU, NUO, UDERO> Mult_AnXBn_Synch(SpParMat<IU, NU1, UDERA>& A, SpParMat<IU, NU2, UDERB>& B,
                                          bool clearA = false, bool clearB = false) {
  constexpr bool dev = DeviceSemiring<SR>::ok && DeviceType<NUO>::ok &&
                       (std::is_same<NU1, NUO>::value || std::is_same<NU1, bool>::value) &&
                       (std::is_same<NU2, NUO>::value || std::is_same<NU2, bool>::value);
  if constexpr (!dev) return combblas::Mult_AnXBn_Synch<SR, NUO, UDERO>(A, B, clearA, clearB);
  else return summa2d<SR, NUO, UDERO>(A, B, clearA, clearB, 0u);
}

template <class SR, class NUO, class UDERO, class IU, class NU1, class NU2, class UDERA, class UDERB>
SpParMat<IU, NUO, UDERO> Mult_AnXBn_DoubleBuff(SpParMat<IU, NU1, UDERA>& A, SpParMat<IU, NU2, UDERB>& B,
                                               bool clearA = false, bool clearB = false) {
  constexpr bool dev = DeviceSemiring<SR>::ok && DeviceType<NUO>::ok &&
                       (std::is_same<NU1, NUO>::value || std::is_same<NU1, bool>::value) &&
                       (std::is_same<NU2, NUO>::value || std::is_same<NU2, bool>::value);
  if constexpr (!dev) return combblas::Mult_AnXBn_DoubleBuff<SR, NUO, UDERO>(A, B, clearA, clearB);
  else return summa2d<SR, NUO, UDERO>(A, B, clearA, clearB, CBG_HALVES);
}

template <class SR, class NUO, class UDERO, class IU, class NU1, class NU2, class UDERA, class UDERB>
SpParMat<IU, NUO, UDERO> Mult_AnXBn_Overlap(SpParMat<IU, NU1, UDERA>& A, SpParMat<IU, NU2, UDERB>& B,
                                            bool clearA = false, bool clearB = false) {
  constexpr bool dev = DeviceSemiring<SR>::ok && DeviceType<NUO>::ok &&
                       (std::is_same<NU1, NUO>::value || std::is_same<NU1, bool>::value) &&
                       (std::is_same<NU2, NUO>::value || std::is_same<NU2, bool>::value);
  if constexpr (!dev) return combblas::Mult_AnXBn_Overlap<SR, NUO, UDERO>(A, B, clearA, clearB);
  else return summa2d<SR, NUO, UDERO>(A, B, clearA, clearB, CBG_RUNNING_MERGE);
}

// PSpGEMM (SpParMat.h:451-464): the default distributed product, Mult_AnXBn_Synch
template <typename SR, typename IU, typename NU1, typename NU2, typename UDERA, typename UDERB>
SpParMat<IU, typename promote_trait<NU1, NU2>::T_promote,
         typename promote_trait<UDERA, UDERB>::T_promote>
PSpGEMM(SpParMat<IU, NU1, UDERA>& A, SpParMat<IU, NU2, UDERB>& B, bool clearA = false, bool clearB = false) {
  typedef typename promote_trait<NU1, NU2>::T_promote N_promote;
  typedef typename promote_trait<UDERA, UDERB>::T_promote DER_promote;
  return gpu::Mult_AnXBn_Synch<SR, N_promote, DER_promote>(A, B, clearA, clearB);
}

// Mult_AnXBn_SUMMA3D on the reference's (non-special) SpParMat3D layout: A colsplit, B rowsplit
template <class SR, class NUO, class UDERO, class IU, class NU1, class NU2, class UDER1, class UDER2>
SpParMat3D<IU, NUO, UDERO> Mult_AnXBn_SUMMA3D(SpParMat3D<IU, NU1, UDER1>& A, SpParMat3D<IU, NU2, UDER2>& B) {
  constexpr bool dev = DeviceSemiring<SR>::ok && DeviceType<NUO>::ok &&
                       (std::is_same<NU1, NUO>::value || std::is_same<NU1, bool>::value) &&
                       (std::is_same<NU2, NUO>::value || std::is_same<NU2, bool>::value);
  if constexpr (!dev) {
    return combblas::Mult_AnXBn_SUMMA3D<SR, NUO, UDERO>(A, B);
  } else {
    std::shared_ptr<CommGrid3D> G = A.getcommgrid3D();
    if (A.getncol() != B.getnrow() || !A.isColSplit() || B.isColSplit() || A.isSpecial() || B.isSpecial())
      throw std::runtime_error("Mult_AnXBn_SUMMA3D: needs colsplit A, rowsplit B, non-special layout (3002)");
    std::shared_ptr<CommGrid> layer = G->GetCommGridLayer();
    cbg_grid* grid = cached_grid(G->GetWorld(), layer->GetRowWorld(), layer->GetColWorld(), G->GetFiberWorld(),
                                 G->GetGridLayers(), G->GetGridRows(), G->GetGridCols());
    cbg_dcsc_view va = view_of(*A.seqptr()), vb = view_of(*B.seqptr());
    cbg_csc_result C{};
    cbg_grid_stats st{};
    check(cbg_spgemm_grid(grid, &va, &vb, DeviceSemiring<SR>::code, DeviceType<NUO>::code, CBG_SORTED_COLS, &C, &st),
          "cbg_spgemm_grid");
    UDERO* D = to_local<IU, NUO, UDERO>(C);
    return SpParMat3D<IU, NUO, UDERO>(D, G, true, false);
  }
}

#ifdef _CC_GRID_
// ------------------------------------------------------------ 3DSpGEMM (split-3D driver of 2015)
// CCGrid (3DSpGEMM/CCGrid.h:9-30) numbers ranks layer-fastest; its rowWorld / colWorld / fiberWorld are
// ordered by proc column / proc row / layer, which are the library's member indices of ROW / COL / FIBER.
// splitA = A[row block i, layer-l part of column block j], splitB = B[layer-l part of row block i, column
// block j] (SplitMat, SplitMatDist.h:143-213); the product piece is the layer-l part of C's block (i, j)
// (ParallelReduce_Alltoall_threaded, Reductions.h:36-130).  PlusTimes over NT, as the reference hard-codes.
inline int ccgrid_rank(const CCGrid& CMG) {
  return CMG.layer_grid * CMG.GridRows * CMG.GridCols + CMG.RankInCol * CMG.GridCols + CMG.RankInRow;
}

inline cbg_grid* ccgrid_grid(CCGrid& CMG) {
  if (CMG.GridRows != CMG.GridCols) throw std::runtime_error("3DSpGEMM: square layer grid required (3002)");
  return cached_grid(MPI_COMM_WORLD, CMG.rowWorld, CMG.colWorld, CMG.fiberWorld, CMG.GridLayers, CMG.GridRows,
                     CMG.GridCols, ccgrid_rank(CMG));
}

// isBT: splitB holds B's piece locally transposed ("outer" mode of test_mpipspgemm.cpp:101-117)
template <typename IT, typename NT>
cbg_dcsc_view b_view(SpDCCols<IT, NT>& splitB, bool isBT, std::unique_ptr<SpDCCols<IT, NT>>& tmp) {
  if (!isBT) return view_of(splitB);
  tmp.reset(new SpDCCols<IT, NT>(splitB));
  tmp->Transpose();
  return view_of(*tmp);
}

// SUMMALayer (SUMMALayer.h:24-97): the q stage products of this rank's layer, unmerged, in stage order
template <typename IT, typename NT>
void SUMMALayer(SpDCCols<IT, NT>& SplitA, SpDCCols<IT, NT>& SplitB, std::vector<SpTuples<IT, NT>*>& C, CCGrid& CMG,
                bool isBT, bool threaded) {
  static_assert(DeviceType<NT>::ok, "3DSpGEMM on the device: NT must be a device value type");
  (void)threaded;   // LocalSpGEMM vs MultiplyReturnTuples is a CPU choice: one device product
  cbg_grid* grid = ccgrid_grid(CMG);
  std::unique_ptr<SpDCCols<IT, NT>> bt;
  cbg_dcsc_view va = view_of(SplitA), vb = b_view(SplitB, isBT, bt);
  std::vector<cbg_csc_result> parts(2 * CMG.GridCols + 2);
  int32_t n = 0;
  cbg_grid_stats st{};
  check(cbg_summa_layer(grid, &va, &vb, CBG_SR_PLUS_TIMES, DeviceType<NT>::code, CBG_SORTED_COLS, parts.data(), &n,
                        &st), "cbg_summa_layer");
  for (int32_t k = 0; k < n; ++k) C.push_back(to_tuples<IT, NT>(context(), parts[k]));
}

// multiply (Multiplier.h:10-61) = SUMMALayer + ReduceAll_threaded, run as one device product
template <typename IT, typename NT>
SpDCCols<IT, NT>* multiply(SpDCCols<IT, NT>& splitA, SpDCCols<IT, NT>& splitB, CCGrid& CMG, bool isBT, bool threaded) {
  static_assert(DeviceType<NT>::ok, "3DSpGEMM on the device: NT must be a device value type");
  (void)threaded;
  cbg_grid* grid = ccgrid_grid(CMG);
  std::unique_ptr<SpDCCols<IT, NT>> bt;
  cbg_dcsc_view va = view_of(splitA), vb = b_view(splitB, isBT, bt);
  cbg_csc_result C{};
  cbg_grid_stats st{};
  check(cbg_spgemm_grid(grid, &va, &vb, CBG_SR_PLUS_TIMES, DeviceType<NT>::code, CBG_SORTED_COLS, &C, &st),
        "cbg_spgemm_grid");
  SpTuples<IT, NT>* t = to_tuples<IT, NT>(context(), C);
  SpDCCols<IT, NT>* D = new SpDCCols<IT, NT>(*t, false);
  delete t;
  return D;
}

// RestrictionOp (3DSpGEMM/RestrictionOp.h:196-291): layer 0 builds R and R^T of the layer's matrix.  The layer's
// pieces are gathered on its rank 0, the device computes the reference's ONE-rank R there (cbg_restriction_op:
// MIS2 on the MTRand stream, Select2ndRandSR, RandPerm; the reference's DETERMINISTIC seeds by default) and every
// rank of layer 0 receives its block of R (n x nagg) and R^T in the SpParMat block distribution of the layer grid
// (RestrictionOp.h:287-288 keep Rop.seq()).  The reference's own R depends on its rank count (each rank draws its
// part of the stream), so at one rank per layer the two are equal entry for entry; on a q x q layer this returns
// the one-rank R.  Values are 1.
template <typename IT, typename NT>
void RestrictionOp(CCGrid& CMG, SpDCCols<IT, NT>* localmat, SpDCCols<IT, NT>*& R, SpDCCols<IT, NT>*& RT,
                   uint32_t mt_seed = 1, uint32_t perm_seed = 1383098845) {
  if (CMG.layer_grid != 0) return;
  MPI_Comm lw = CMG.layerWorld;
  int lr = 0, ls = 1;
  MPI_Comm_rank(lw, &lr);
  MPI_Comm_size(lw, &ls);
  const int q = CMG.GridCols, bi = lr / q, bj = lr % q;
  // the layer matrix's size and this piece's offsets (colWorld orders the grid column by row, rowWorld the grid
  // row by column)
  int64_t m = localmat->getnrow(), n = localmat->getncol(), M = 0, N = 0, roff = 0, coff = 0;
  MPI_Allreduce(&m, &M, 1, MPI_INT64_T, MPI_SUM, CMG.colWorld);
  MPI_Allreduce(&n, &N, 1, MPI_INT64_T, MPI_SUM, CMG.rowWorld);
  MPI_Exscan(&m, &roff, 1, MPI_INT64_T, MPI_SUM, CMG.colWorld);
  MPI_Exscan(&n, &coff, 1, MPI_INT64_T, MPI_SUM, CMG.rowWorld);
  if (bi == 0) roff = 0;
  if (bj == 0) coff = 0;
  if (M != N) throw std::runtime_error("RestrictionOp: square matrix required (3002)");
  // the pattern's global (row, col) pairs on the layer's rank 0
  std::vector<int64_t> mine;
  {
    SpTuples<IT, NT> T(*localmat);
    mine.resize(2 * (size_t)T.getnnz());
    for (int64_t k = 0; k < T.getnnz(); ++k) {
      mine[2 * k] = (int64_t)T.rowindex(k) + roff;
      mine[2 * k + 1] = (int64_t)T.colindex(k) + coff;
    }
  }
  int cnt = (int)mine.size();
  std::vector<int> cnts(ls), displs(ls + 1, 0);
  MPI_Gather(&cnt, 1, MPI_INT, cnts.data(), 1, MPI_INT, 0, lw);
  for (int r = 0; r < ls; ++r) displs[r + 1] = displs[r] + cnts[r];
  std::vector<int64_t> all(lr == 0 ? (size_t)displs[ls] : 0);
  MPI_Gatherv(mine.data(), cnt, MPI_INT64_T, all.data(), cnts.data(), displs.data(), MPI_INT64_T, 0, lw);
  int64_t nagg = 0;
  std::vector<int64_t> agg;   // aggregate (column of R) of every vertex, on rank 0
  std::string err;            // rank 0's failure, broadcast as a status so every rank throws together
  if (lr == 0) try {
    const int64_t nnz = (int64_t)all.size() / 2;
    std::vector<int64_t> cp((size_t)N + 1, 0);
    for (int64_t k = 0; k < nnz; ++k) cp[(size_t)all[2 * k + 1] + 1]++;
    for (int64_t c = 0; c < N; ++c) cp[(size_t)c + 1] += cp[(size_t)c];
    std::vector<int32_t> ir((size_t)nnz + 1);
    std::vector<int64_t> cur(cp.begin(), cp.end() - 1);
    for (int64_t k = 0; k < nnz; ++k) ir[(size_t)cur[(size_t)all[2 * k + 1]]++] = (int32_t)all[2 * k];
    for (int64_t c = 0; c < N; ++c) std::sort(ir.begin() + cp[(size_t)c], ir.begin() + cp[(size_t)c + 1]);
    cbg_dcsc_view v{};
    v.nrow = M; v.ncol = N; v.nnz = nnz; v.nzc = N;
    v.cp = cp.data(); v.jc = nullptr; v.ir = ir.data(); v.idx_bytes = 4; v.ptr_bytes = 8;
    v.val = nullptr; v.val_type = CBG_F64; v.on_device = 0;
    cbg_csc_result Rd{}, RTd{};
    check(cbg_restriction_op(context(), &v, mt_seed, perm_seed, &Rd, &RTd, &nagg), "cbg_restriction_op");
    // R^T has one entry per column: its rows are the aggregates of the vertices
    std::vector<int64_t> tcp((size_t)M + 1);
    std::vector<int32_t> trow((size_t)M + 1);
    std::vector<double> tval((size_t)M + 1);
    check(cbg_result_to_host(context(), &RTd, tcp.data(), trow.data(), tval.data()), "cbg_result_to_host");
    cbg_result_free(context(), &Rd);
    cbg_result_free(context(), &RTd);
    agg.assign(trow.begin(), trow.begin() + M);
  } catch (std::exception& e) {
    err = e.what();
  }
  int failed = !err.empty();
  MPI_Bcast(&failed, 1, MPI_INT, 0, lw);
  if (failed) throw std::runtime_error(lr == 0 ? err : std::string("RestrictionOp failed on the layer's rank 0"));
  MPI_Bcast(&nagg, 1, MPI_INT64_T, 0, lw);
  agg.resize((size_t)M);
  MPI_Bcast(agg.data(), (int)M, MPI_INT64_T, 0, lw);
  // blocks of the SpParMat distribution on the q x q layer grid: n / q per block, the last takes the remainder
  auto blk = [q](int64_t len, int b, int64_t* lo, int64_t* hi) {
    *lo = (len / q) * b;
    *hi = b == q - 1 ? len : (len / q) * (b + 1);
  };
  int64_t r0, r1, c0, c1;
  blk(M, bi, &r0, &r1);      // R: rows = vertices, cols = aggregates
  blk(nagg, bj, &c0, &c1);
  std::vector<std::tuple<IT, IT, NT>> tr, tt;
  for (int64_t v = r0; v < r1; ++v)
    if (agg[(size_t)v] >= c0 && agg[(size_t)v] < c1)
      tr.emplace_back((IT)(v - r0), (IT)(agg[(size_t)v] - c0), (NT)1);
  int64_t t0, t1, u0, u1;
  blk(nagg, bi, &t0, &t1);   // R^T: rows = aggregates, cols = vertices
  blk(M, bj, &u0, &u1);
  for (int64_t v = u0; v < u1; ++v)
    if (agg[(size_t)v] >= t0 && agg[(size_t)v] < t1)
      tt.emplace_back((IT)(agg[(size_t)v] - t0), (IT)(v - u0), (NT)1);
  auto build = [](std::vector<std::tuple<IT, IT, NT>>& t, int64_t nr, int64_t nc) {
    std::tuple<IT, IT, NT>* a = new std::tuple<IT, IT, NT>[t.size() > 0 ? t.size() : 1];
    std::copy(t.begin(), t.end(), a);
    SpTuples<IT, NT> T((IT)t.size(), (IT)nr, (IT)nc, a, false, false);
    T.SortColBased();
    return new SpDCCols<IT, NT>(T, false);
  };
  R = build(tr, r1 - r0, c1 - c0);
  RT = build(tt, t1 - t0, u1 - u0);
}
#endif  // _CC_GRID_

}  // namespace gpu
}  // namespace combblas

#endif  // COMBBLAS_GPU_H
