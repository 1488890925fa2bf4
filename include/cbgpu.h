/*
 * cbgpu.h -- C ABI of the MI355X-native CombBLAS SpGEMM path (libcbgpu.so).
 *
 * Plain C: POD structs, raw pointers and sizes, no C++/torch types.  Every entry point is the
 * device replacement of one reference interface (file:line under gabe-raulet/CombBLAS):
 *
 *   cbg_spgemm_local   LocalSpGEMMHash<SR,NTO>(A,B,clearA,clearB,sort)  include/CombBLAS/mtSpGEMM.h:465-470
 *                      LocalHybridSpGEMM<SR,NTO>(A,B,clearA,clearB,aux)  include/CombBLAS/mtSpGEMM.h:212-217
 *                      LocalSpGEMM<SR,NTO>(A,B,clearA,clearB)            include/CombBLAS/mtSpGEMM.h:73-78
 *   cbg_estimate       estimateFLOP + estimateNNZ_Hash                   include/CombBLAS/mtSpGEMM.h:1061-1139, 810-938
 *                      EstimateLocalFLOP                                 include/CombBLAS/mtSpGEMM.h:667-694
 *   cbg_merge          MultiwayMerge<SR>(lists, m, n, delarrs)           include/CombBLAS/MultiwayMerge.h:411-412
 *                      MultiwayMergeHash<SR>(lists, m, n, delarrs, sorted) include/CombBLAS/MultiwayMerge.h:536-537
 *   cbg_generate_rmat  DistEdgeList::GenGraph500Data + SpParMat(DEL)     include/CombBLAS/DistEdgeList.cpp:223-280,
 *   cbg_rmat_block     (+ RefGen21 edge stream, SpTuples dup-summing)    include/CombBLAS/SpParMat.cpp:3082-3196,
 *                                                                        RefGen21.h:102-318, SpTuples.cpp:66-115
 *   cbg_mcl_prune      MCLPruneRecoverySelect(A, thr, select, recover, pct, kselectVersion)
 *                                                                        include/CombBLAS/ParFriends.h:185-353
 *                      (Kselect1 SpParMat.cpp:1413-1700, PruneColumn SpParMat.cpp:2567-2720)
 *   cbg_mis2_restriction MIS2 + RestrictionOp                            3DSpGEMM/RestrictionOp.h:116-290
 *   cbg_galerkin_rap   R^T A R (RestrictionOp.cpp:188-196's two products, fused for aggregation R)
 *   cbg_col_range      SpDCCols::ColSplit (one piece)                    include/CombBLAS/SpDCCols.cpp:927-1086
 *   cbg_col_concat     SpDCCols::ColConcatenate                          include/CombBLAS/SpDCCols.cpp:1087-1185
 *   cbg_col_select     SubsRef_SR column form on one block               include/CombBLAS/SpParMat.cpp:2251-2422
 *   cbg_spgemm_grid    Mult_AnXBn_Synch / PSpGEMM / DoubleBuff / Overlap include/CombBLAS/ParFriends.h:798-1235
 *                      Mult_AnXBn_SUMMA3D                                include/CombBLAS/ParFriends.h:2918-3208
 *   cbg_summa_layer    SUMMALayer                                        3DSpGEMM/SUMMALayer.h:24-97
 *   cbg_reduce_all     ReduceAll_threaded                                3DSpGEMM/Reductions.h:134-155
 *   cbg_grid_create*   CommGrid / CommGrid3D / CCGrid                    src/CommGrid.cpp:37-76, CommGrid3D.h:21-80
 *
 * Semantics (SURVEY §8a parity rules):
 *   - Output columns are row-sorted and duplicate-free when CBG_SORTED_COLS is set (the reference
 *     intends this but its integerSort mis-sorts, PBBS/radixSort.h:116-120; we sort correctly).
 *   - Entries whose value equals the semiring zero are kept (returnedSAID() is always false).
 *   - SELECT2ND keeps the product of the first contributing B nonzero in storage order
 *     (mtSpGEMM.h:583: SR::add(new, existing) returns `existing`).
 *   - BOOL_COPY1ST/2ND: a second contribution to one output entry is an error (the reference's
 *     add() throws, Semirings.h:55-60, 101-106) -> CBG_EADD.
 *   - Errors never abort the process: DIMMISMATCH (SpDefs.h:73) is returned as CBG_EDIM, etc.
 *
 * Memory: views are borrowed (clearA/clearB ownership transfer stays with the C++ caller).
 * Results are owned by the library until cbg_result_free.  Device pointers are HIP device
 * pointers on the context's device; host views are staged to the device by the library.
 */
#ifndef CBGPU_H
#define CBGPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CBG_ABI_VERSION 4   /* 2: cbg_grid_stats.fiber_xfer_ms after stages; cbg_device_count
                               3: cbg_profile heavy_* counts; cbg_grid_stats heavy / local-product sums;
                                  cbg_fiber_codec
                               4: cbg_grid_stats.fiber_mode */

typedef enum {
  CBG_OK = 0,
  CBG_EDIM = 3002,      /* DIMMISMATCH, SpDefs.h:73 */
  CBG_EALIAS = 3005,    /* MATRIXALIAS, SpDefs.h:76 */
  CBG_ENOMEM = 10,
  CBG_EUNSUP = 11,      /* semiring/dtype combination without a device functor */
  CBG_EDEVICE = 12,     /* HIP runtime error, or no GPU */
  CBG_EADD = 13,        /* BoolCopy1st/2nd add() would have been called */
  CBG_EINVAL = 14,      /* malformed view (bad idx_bytes, NULL arrays with nnz>0, ...) */
  CBG_ECOMM = 15        /* RCCL error */
} cbg_status;

typedef enum {
  CBG_SR_PLUS_TIMES = 0,      /* PlusTimesSRing, Semirings.h:212-233 */
  CBG_SR_MIN_PLUS = 1,        /* MinPlusSRing + inf_plus, Semirings.h:235-255, 40-47 */
  CBG_SR_SELECT2ND = 2,       /* Select2ndSRing, Semirings.h:143-163 */
  CBG_SR_SELECT_MAX = 3,      /* SelectMaxSRing<T1,T2>, Semirings.h:165-190 */
  CBG_SR_SELECT_MAX_BOOL = 4, /* SelectMaxSRing<bool,T2>, Semirings.h:191-210 (A is a pattern) */
  CBG_SR_BOOL_COPY1ST = 5,    /* BoolCopy1stSRing, Semirings.h:96-141 (B is a pattern) */
  CBG_SR_BOOL_COPY2ND = 6     /* BoolCopy2ndSRing, Semirings.h:50-94 (A is a pattern) */
} cbg_semiring;

typedef enum { CBG_BOOL = 0, CBG_I32 = 1, CBG_I64 = 2, CBG_F32 = 3, CBG_F64 = 4 } cbg_dtype;

/* flags for cbg_spgemm_local / cbg_merge */
#define CBG_SORTED_COLS 1u     /* row-sort every output column (LocalSpGEMMHash sort=true) */
#define CBG_KEEP_ON_DEVICE 2u  /* leave the result on device only (no host mirror) */

/*
 * Borrowed view of a local matrix: either a CSC (nzc == ncol, jc == NULL, cp dense ncol+1) or the
 * reference's DCSC (Dcsc: cp[nzc+1], jc[nzc], ir[nnz], numx[nnz]; dcsc.h:123-130), i.e. exactly the
 * arrays SpDCCols::GetArrays() hands out (SpDCCols.cpp:817-839).  Row indices ascend within a column.
 */
typedef struct {
  int64_t nrow, ncol, nnz, nzc;
  const void* cp;       /* nzc+1 entries of ptr_bytes */
  const void* jc;       /* nzc entries of idx_bytes, or NULL for CSC */
  const void* ir;       /* nnz entries of idx_bytes */
  int32_t idx_bytes;    /* 4 or 8: row (ir) and column-id (jc) index width (the reference's IT) */
  int32_t ptr_bytes;    /* 4 or 8: column pointer (cp) width; 0 = same as idx_bytes */
  const void* val;      /* nnz values of val_type, or NULL for a pattern (all true / 1) */
  cbg_dtype val_type;
  int32_t on_device;    /* 1: HIP device pointers, 0: host pointers */
} cbg_dcsc_view;

/* Result: CSC with dense colptr (ncol+1). Device arrays always valid; host mirror unless KEEP_ON_DEVICE. */
typedef struct {
  int64_t nrow, ncol, nnz;
  int64_t* colptr;      /* device, ncol+1 */
  int32_t* row;         /* device, nnz */
  void* val;            /* device, nnz of val_type */
  cbg_dtype val_type;
  int64_t multiplies;   /* estimateFLOP total of the product that made it */
  void* _owner;         /* library-internal */
} cbg_csc_result;

typedef struct cbg_ctx cbg_ctx;

/* Per-phase device times (ms) of the last call on a context, from HIP events. */
typedef struct {
  double flops_ms, bin_ms, symbolic_ms, scan_ms, numeric_ms, total_ms;
  int64_t multiplies, nnz_out, bins[16];
  double heavy_ms;      /* k_num_heavy_known + k_num_heavy (heavy-column units), HIP events on the context stream */
  int64_t known_items;  /* heavy units whose rows came from the symbolic pass (k_num_heavy_known) */
  /* ABI 3: what the heavy kernels processed (columns with nnz(C(:,j)) > 4096): multiplies, B nonzeros, outputs --
   * the per-unit counts of SURVEY 8(d)'s algorithmic bytes of the dominant kernels */
  int64_t heavy_multiplies, heavy_nnz_b, heavy_nnz_c;
} cbg_profile;

int32_t     cbg_abi_version(void);
const char* cbg_strerror(cbg_status s);

/* Number of visible HIP devices (the C++ drop-in binds MPI rank r to device node-local-rank % count). */
cbg_status cbg_device_count(int32_t* n);
cbg_status cbg_init(int device, cbg_ctx** ctx);
cbg_status cbg_destroy(cbg_ctx* ctx);
/* Use an external HIP stream (hipStream_t) for all subsequent work on ctx; NULL = own stream. */
cbg_status cbg_set_stream(cbg_ctx* ctx, void* hip_stream);
cbg_status cbg_synchronize(cbg_ctx* ctx);

/* C = A (x) B over the semiring.  out_type is the value type A, B and C are computed in. */
cbg_status cbg_spgemm_local(cbg_ctx* ctx, const cbg_dcsc_view* A, const cbg_dcsc_view* B,
                            cbg_semiring sr, cbg_dtype out_type, uint32_t flags,
                            cbg_csc_result* C, int64_t* multiplies_out);

/* Symbolic only: total multiplies (estimateFLOP) and exact nnz(C) (estimateNNZ_Hash).
 * per-column arrays are optional device or host pointers (on_device of B) of length ncol(B). */
cbg_status cbg_estimate(cbg_ctx* ctx, const cbg_dcsc_view* A, const cbg_dcsc_view* B,
                        int64_t* multiplies, int64_t* nnz_c);

/* Merge nparts column-sorted partial products of identical shape; duplicates combined with
 * SR::add in part order, MultiwayMergeHash's order (SerialMergeHash, MultiwayMerge.h:320-405:
 * for Select2nd the first part holding an entry wins; the heap MultiwayMerge differs only there,
 * tests/golden/merge.npz pins both). */
cbg_status cbg_merge(cbg_ctx* ctx, const cbg_csc_result* parts, int32_t nparts, cbg_semiring sr,
                     cbg_dtype val_type, uint32_t flags, cbg_csc_result* C);

/* Copy a result to caller-owned arrays (colptr ncol+1, row nnz, val nnz), host or device memory
 * (unified addressing; a device destination stays a device-to-device copy). */
cbg_status cbg_result_to_host(cbg_ctx* ctx, const cbg_csc_result* C, int64_t* colptr, int32_t* row,
                              void* val);
void       cbg_result_free(cbg_ctx* ctx, cbg_csc_result* C);

/* Device-resident CSC owned by the library (inputs kept in HBM across calls, e.g. for benches). */
cbg_status cbg_upload(cbg_ctx* ctx, const cbg_dcsc_view* host, cbg_csc_result* dev);
/* A view of a library-owned device CSC, usable as an input of cbg_spgemm_local. */
cbg_status cbg_result_view(const cbg_csc_result* C, cbg_dcsc_view* view);

cbg_status cbg_last_profile(cbg_ctx* ctx, cbg_profile* prof);

/* Host-only CSC (malloc'd by the library, freed with cbg_host_free). */
typedef struct {
  int64_t nrow, ncol, nnz;
  int64_t* colptr;
  int32_t* row;
  double* val;
} cbg_host_csc;

/*
 * Graph500 Kronecker/R-MAT input exactly as the reference builds it for its R-MAT runs:
 * DistEdgeList::GenGraph500Data(initiator .57/.19/.19/.05, scale, edgefactor, scramble, packed)
 * (DistEdgeList.cpp:223-280, RefGen21.h:102-318: MRG stream, clip-and-flip, scrambled vertex ids)
 * then SpParMat(DistEdgeList, removeloops=false) (SpParMat.cpp:3082-3196): edge (v0, v1) -> A(v0, v1),
 * duplicate edges summed into the value = multiplicity (f64), loops kept.  `seed` is the Graph500
 * user seed (the reference's SEED environment variable, default 0xDECAFBAD, RefGen21.h:306-318).
 *
 * cbg_rmat_block: the block rows [r0, r1) x cols [c0, c1) of that matrix (local indices), built on
 *   the device: every rank replays the edge stream and keeps its own block (no communication).
 * cbg_generate_rmat: the whole matrix on the device.
 * cbg_rmat_host: the whole matrix built on the host only (no GPU needed).
 */
cbg_status cbg_rmat_block(cbg_ctx* ctx, int32_t scale, int32_t edgefactor, uint64_t seed, int64_t r0, int64_t r1,
                          int64_t c0, int64_t c1, cbg_csc_result* A);
cbg_status cbg_generate_rmat(cbg_ctx* ctx, int32_t scale, int32_t edgefactor, uint64_t seed,
                             cbg_csc_result* A);
cbg_status cbg_rmat_host(int32_t scale, int32_t edgefactor, uint64_t seed, cbg_host_csc* out);
void       cbg_host_free(cbg_host_csc* m);

/*
 * HipMCL expansion support (MemEfficientSpGEMM, ParFriends.h:449-730).
 *
 * cbg_mcl_prune: per column of a column-complete local matrix (every row of each column present,
 * e.g. a 1-rank product or a column-gathered piece), exactly MCLPruneRecoverySelect's rule:
 *   P = {v > hardThreshold}; recover if |P| < recoverNum && nnz > |P| && sum(P) < recoverPct
 *   (threshold = recoverNum-th largest); else select if selectNum > 0 && |P| > selectNum
 *   (threshold = selectNum-th largest, then recovery-after-selection as ParFriends.h:290-333);
 *   else threshold = hardThreshold.  Entries v < threshold are dropped (PruneColumn with less<>).
 * k-th largest follows Kselect1: fewer than k entries -> the column minimum.  Values f32/f64.
 * The output is a new library-owned result (same nrow/ncol); row order within columns is kept.
 */
typedef struct {
  int64_t recovered;               /* columns taking the recovery branch */
  int64_t selected;                /* columns taking the selection branch */
  int64_t recovered_after_select;  /* selected columns recovered again */
  int64_t nnz_in, nnz_out;
} cbg_mcl_stats;

cbg_status cbg_mcl_prune(cbg_ctx* ctx, const cbg_csc_result* in, double hardThreshold, int64_t selectNum,
                         int64_t recoverNum, double recoverPct, cbg_csc_result* out, cbg_mcl_stats* stats);
/* Columns [c0, c1) of a device CSC as a new result (colptr rebased).  c out of range -> CBG_EDIM. */
cbg_status cbg_col_range(cbg_ctx* ctx, const cbg_csc_result* in, int64_t c0, int64_t c1, cbg_csc_result* out);
/* Columns cols[0..ncols) (host array, any order, repeats allowed) of a device CSC as a new result:
 * the column form of SpParMat::SubsRef_SR (A(:, ci), SpParMat.cpp:2251-2422) on one block.
 * A column id out of range -> CBG_EDIM. */
cbg_status cbg_col_select(cbg_ctx* ctx, const cbg_csc_result* in, const int64_t* cols, int64_t ncols,
                          cbg_csc_result* out);
/* Horizontal concatenation of nparts device CSCs with equal nrow/val_type. */
cbg_status cbg_col_concat(cbg_ctx* ctx, const cbg_csc_result* parts, int32_t nparts, cbg_csc_result* out);

/*
 * Galerkin coarse operator (BASELINE config 5; 3DSpGEMM/RestrictionOp.h:116-290, RestrictionOp.cpp:155-196).
 *
 * cbg_mis2_restriction: MIS-2 of the graph G (square, symmetric, pattern; self loops ignored) by Luby
 *   rounds with seeded distinct priorities, then every vertex joins the highest-priority set vertex
 *   within distance 1, else 2: R (n x nagg, R(i, agg(i)) = 1, columns row-sorted) and, if RT is not
 *   NULL, R^T (nagg x n).  Aggregates are numbered in the order of their root vertices.
 * cbg_galerkin_rap: C = R^T A R in one pass for an aggregation R (exactly one nonzero per row of R, any
 *   value; otherwise CBG_EUNSUP -- use two cbg_spgemm_local products), PlusTimes<double>, row-sorted.
 *   C.multiplies = nnz(A) (one scaled copy per nonzero of A).
 */
cbg_status cbg_mis2_restriction(cbg_ctx* ctx, const cbg_dcsc_view* G, uint64_t seed, cbg_csc_result* R,
                                cbg_csc_result* RT, int64_t* nagg);
/*
 * cbg_restriction_op: the reference's RestrictionOp (3DSpGEMM/RestrictionOp.h:196-291) of the square matrix A
 *   (values ignored) at one rank, entry for entry: B = pattern(A) + pattern(A)^T without loops, MIS2 on B
 *   (:116-193) with the MTRand stream of mt_seed, parents by MIS2verifySR, one draw per parented vertex,
 *   Select2ndRandSR for the rest (equal draws: the larger neighbour), aggregate columns in set-vertex order
 *   permuted by RandPerm (std::shuffle, std::default_random_engine(perm_seed); FullyDistVec.cpp:783-900).
 *   The reference's DETERMINISTIC seeds are mt_seed = 1, perm_seed = 1383098845 (its output is deterministic
 *   with one OpenMP thread only).  R (n x nagg, R(i, agg(i)) = 1) and, if RT is not NULL, R^T.
 */
cbg_status cbg_restriction_op(cbg_ctx* ctx, const cbg_dcsc_view* A, uint32_t mt_seed, uint32_t perm_seed,
                              cbg_csc_result* R, cbg_csc_result* RT, int64_t* nagg);
cbg_status cbg_galerkin_rap(cbg_ctx* ctx, const cbg_dcsc_view* A, const cbg_dcsc_view* R, cbg_csc_result* C);
/* C = A^T (SpDCCols::Transpose, SpDCCols.cpp:845) on the device, rows sorted; f64 values or a pattern. */
cbg_status cbg_transpose(cbg_ctx* ctx, const cbg_dcsc_view* A, cbg_csc_result* C);

/*
 * ---------------------------------------------------------------------------------------------
 * Distributed SpGEMM on a layers x rows x cols process grid, one process (rank) per GPU.
 *
 *   cbg_grid_create_rccl / cbg_grid_create   CommGrid3D(world, nlayers, rows, cols)
 *                                            include/CombBLAS/CommGrid3D.h:21-80 (CommGrid, src/CommGrid.cpp:37-76)
 *   cbg_spgemm_grid    Mult_AnXBn_SUMMA3D(A3D, B3D)              include/CombBLAS/ParFriends.h:2918-3208
 *                      Mult_AnXBn_Synch / PSpGEMM (one layer)     ParFriends.h:1004-1108, SpParMat.h:451-464
 *                      Mult_AnXBn_DoubleBuff (CBG_HALVES)         ParFriends.h:798-997
 *                      Mult_AnXBn_Overlap (CBG_RUNNING_MERGE)     ParFriends.h:1110-1235
 *   cbg_summa_layer    SUMMALayer(splitA, splitB, unreducedC, CMG) 3DSpGEMM/SUMMALayer.h:24-97
 *   cbg_reduce_all     ReduceAll_threaded(unreducedC, CMG)        3DSpGEMM/Reductions.h:134-155
 *                      (multiply() = SUMMALayer + ReduceAll_threaded, 3DSpGEMM/Multiplier.h:10-61)
 *
 * Rank r = (l, i, j) with r = l*rows*cols + i*cols + j (CommGrid3D::GetRank, CommGrid3D.h:90-91);
 * rows == cols = q (SUMMA needs a square layer grid, CommGrid.cpp:44-50).  Groups, members in
 * increasing rank order: ROW = {(l,i,*)} (member index j), COL = {(l,*,j)} (member i), FIBER =
 * {(*,i,j)} (member l), WORLD (member r).  Layout (SpParMat3D, non-special, SpParMat3D.cpp:337-444):
 * the inner dimension's block k is cut into L layer parts; rank (l,i,j) holds the A piece
 * A[row block i, layer-l part of column block j] ("colsplit") and the B piece B[layer-l part of row
 * block i, column block j] ("rowsplit"); the product's piece comes back colsplit.  Layer l runs q SUMMA stages (stage k: A piece (l,i,k) broadcast along ROW, B piece
 * (l,k,j) along COL: BCastMatrix, SpParHelper.cpp:583-600, sizes exchanged first as GetSetSizes,
 * :798-809), multiplies locally (cbg_spgemm_local) and merges the q partials (cbg_merge); with L > 1
 * the fiber exchanges layer column parts (all-to-all-v, ParFriends.h:3119-3153) and merges them in
 * layer order.  Everything stays in HBM; with RCCL the next stage's broadcasts run on a
 * communication stream while the current stage multiplies.
 *
 * Every call is collective over the grid.  Pieces are views (host or device, CSC or DCSC); results
 * are library-owned device CSCs (cbg_result_free).
 */
typedef enum { CBG_GROUP_ROW = 0, CBG_GROUP_COL = 1, CBG_GROUP_FIBER = 2, CBG_GROUP_WORLD = 3 } cbg_group;

/* Caller-provided transport (e.g. MPI on the reference side, gloo in tests).  bcast / alltoallv get
 * DEVICE buffers of the grid's device (the library has synchronised its streams before the call),
 * or HOST buffers when host_buffers is set (the library stages through host memory: a plain MPI
 * transport); allgather always gets HOST buffers.  root / segment order = member index in the
 * group.  Return 0 on success; anything else makes the library return CBG_ECOMM. */
typedef struct {
  void* user;
  int32_t (*bcast)(void* user, int32_t group, void* buf, int64_t bytes, int32_t root);
  int32_t (*alltoallv)(void* user, int32_t group, const void* send, const int64_t* send_bytes, void* recv,
                       const int64_t* recv_bytes);
  int32_t (*allgather)(void* user, int32_t group, const void* send, void* recv, int64_t bytes);
  int32_t host_buffers;
} cbg_transport;

typedef struct cbg_grid cbg_grid;

/* flags of cbg_spgemm_grid / cbg_summa_layer (besides CBG_SORTED_COLS) */
#define CBG_HALVES 4u          /* Mult_AnXBn_DoubleBuff: operands split in two along the inner dim, 2q stages */
#define CBG_RUNNING_MERGE 8u   /* Mult_AnXBn_Overlap: merge the accumulated product after every stage */

typedef struct {
  int64_t multiplies;          /* this rank's local multiplies */
  int64_t bcast_bytes, fiber_bytes;
  double bcast_ms, local_ms, merge_ms, fiber_ms, total_ms;
  int32_t stages;
  /* ABI 2: fields after `stages` (callers built against ABI 1 never read past it) */
  double fiber_xfer_ms;        /* two layers: the fiber transfer on the communication stream (overlaps local_ms) */
  /* ABI 3: sums over this rank's local products (cbg_profile of each): heavy-kernel time and counts, and the
   * products' outputs / B nonzeros / B columns (SURVEY 8(d) algorithmic bytes of the rank's local work) */
  double heavy_ms;
  int64_t heavy_multiplies, heavy_nnz_b, heavy_nnz_c;
  int64_t local_nnz_out, local_nnz_b, local_ncol_b;
  int32_t local_products;
  /* ABI 4: the two-layer fiber step taken: 0 none (one layer), 1 the reduction of partial products (codec + merge),
   * 2 the gather of the layer operands (one product, no partials) */
  int32_t fiber_mode;
} cbg_grid_stats;

/* RCCL unique id (128 bytes) made on one rank and handed to all (any out-of-band channel). */
cbg_status cbg_rccl_unique_id(char id[128]);
/* Grid over RCCL communicators (world + ncclCommSplit row/col/fiber), on ctx's device and stream. */
cbg_status cbg_grid_create_rccl(cbg_ctx* ctx, const char id[128], int32_t world, int32_t rank, int32_t layers,
                                int32_t rows, int32_t cols, cbg_grid** grid);
/* Grid over a caller-provided transport (copied; `user` must outlive the grid). */
cbg_status cbg_grid_create(cbg_ctx* ctx, const cbg_transport* t, int32_t world, int32_t rank, int32_t layers,
                           int32_t rows, int32_t cols, cbg_grid** grid);
cbg_status cbg_grid_destroy(cbg_grid* grid);
/* What a grid runs over.  rccl = 1: the library's RCCL communicators, ranks[g] = ncclCommCount of the
 * communicator of group g (ROW, COL, FIBER, WORLD; 1 for a group of one, which needs no collective);
 * rccl = 0: a caller transport, ranks[g] = the group sizes. */
typedef struct {
  int32_t rccl;
  int32_t ranks[4];
} cbg_grid_info;
cbg_status cbg_grid_query(const cbg_grid* grid, cbg_grid_info* info);

/* C piece = A (x) B over the grid.  Dimension mismatch on any rank -> CBG_EDIM on every rank. */
cbg_status cbg_spgemm_grid(cbg_grid* grid, const cbg_dcsc_view* A, const cbg_dcsc_view* B, cbg_semiring sr,
                           cbg_dtype out_type, uint32_t flags, cbg_csc_result* C, cbg_grid_stats* stats);
/* The layer SUMMA alone: the unmerged stage products (at most 2*rows entries of `parts`; *nparts set). */
cbg_status cbg_summa_layer(cbg_grid* grid, const cbg_dcsc_view* A, const cbg_dcsc_view* B, cbg_semiring sr,
                           cbg_dtype out_type, uint32_t flags, cbg_csc_result* parts, int32_t* nparts,
                           cbg_grid_stats* stats);
/* EstPerProcessNnzSUMMA (ParFriends.h:1242-1347): the layer SUMMA's broadcasts with only the symbolic pass of
 * every stage product (estimateFLOP + estimateNNZ_Hash); *flops / *nnz are this rank's sums over the stages.
 * No product is formed. */
cbg_status cbg_summa_estimate(cbg_grid* grid, const cbg_dcsc_view* A, const cbg_dcsc_view* B, int64_t* flops,
                              int64_t* nnz);
/* Merge the stage products, then (L > 1) the fiber exchange + merge: the rank's colsplit C piece. */
cbg_status cbg_reduce_all(cbg_grid* grid, const cbg_csc_result* parts, int32_t nparts, cbg_semiring sr,
                          cbg_dtype out_type, cbg_csc_result* C, cbg_grid_stats* stats);

/* ------------------------------------------------------------------ fiber wire codec (test / measurement)
 * The fiber pipeline's production encoder and decoder (grid.hip fiber_pipeline, the wire format of the 3D fiber
 * reduction that replaces ParFriends.h:3119-3153's all-to-all of SpTuples) run on one partial P without a
 * transport: P's columns are cut into `chunks` message chunks as the pipeline cuts them, each chunk is encoded in
 * its smallest lossless form, decoded back, and compared bit for bit with the chunk.  Reports the bytes the
 * messages put on the link (what cbg_grid_stats.fiber_bytes counts in a real exchange). */
typedef struct {
  int64_t columns, entries, chunks;
  int64_t header_bytes, row_bytes, escape_bytes, value_bytes, value_header_bytes, wire_bytes;
  int32_t row_formats;       /* bit f set: some chunk's rows travelled as format f (0 int32, 1 u16 gaps, 2 varint) */
  int32_t value_formats;     /* bit f set: some chunk's values as format f (0 native, 1 f32, 2 u16, 3 varint) */
  int32_t roundtrip_exact;   /* 1: every decoded chunk equals its source (colptr, rows, value bits) */
  int64_t mismatches;        /* entries (or columns) that differ after the round trip */
  double encode_ms, decode_ms;
} cbg_codec_stats;
cbg_status cbg_fiber_codec(cbg_ctx* ctx, const cbg_csc_result* P, int32_t chunks, cbg_codec_stats* stats);

#ifdef __cplusplus
}
#endif
#endif /* CBGPU_H */
