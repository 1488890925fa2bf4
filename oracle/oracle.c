/*
 * oracle/oracle.c -- CPU restatement of CombBLAS's local hash SpGEMM.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  The product
 * path (libcbgpu.so) never links, calls or falls back to it.
 *
 * Pinned against the reference's own outputs: the tests/golden fixtures are produced by
 * oracle/_ref/refprobe (the reference's LocalSpGEMMHash / LocalSpGEMM / Mult_AnXBn_Synch
 * compiled from /root/reference, see oracle/ref/) and by the MATLAB golden
 * 3DSpGEMM/matlab/C.mtx; tests/test_oracle_golden.py checks this restatement against
 * every one of them.
 *
 * Algorithm restated (file:line refer to /root/reference):
 *   orc_flops        estimateFLOP               include/CombBLAS/mtSpGEMM.h:1061-1139
 *   orc_symbolic     estimateNNZ_Hash           include/CombBLAS/mtSpGEMM.h:810-938
 *                    (table = pow2 >= max(16, flop), hash = (key*107) & (size-1),
 *                     linear probing, empty = -1)
 *   orc_spgemm       LocalSpGEMMHash numeric    include/CombBLAS/mtSpGEMM.h:531-642
 *                    (table = pow2 >= max(16, nnzcol), first insert stores the product,
 *                     later hits do val = SR::add(product, val))
 *                    followed by a CORRECT row sort (the reference's PBBS integerSort
 *                    mis-sorts when the column's max row is a power of two,
 *                    include/CombBLAS/PBBS/radixSort.h:116-120).
 *   orc_merge        MultiwayMergeHash order    include/CombBLAS/MultiwayMerge.h:536-684 (SerialMergeHash 320-405);
 *                    = MultiwayMerge (411-526) except Select2nd ties, pinned by tests/golden/merge.npz
 *                    (duplicates combined with SR::add in list order).
 *   orc_mcl_prune    MCLPruneRecoverySelect     include/CombBLAS/ParFriends.h:185-353 on one
 *                    rank (column statistics of Prune(less_equal thr) in storage order,
 *                    Kselect1 SpParMat.cpp:1413-1700: sort descending, k-th item, fewer than
 *                    k -> last item, empty -> numeric_limits<double>::min(); final PruneColumn
 *                    SpParMat.cpp:2567-2720 drops v < threshold).
 * Semirings restate include/CombBLAS/Semirings.h:
 *   PLUS_TIMES 212-233, MIN_PLUS 235-255 (inf_plus 40-47), SELECT2ND 143-163,
 *   SELECT_MAX 165-190, SELECT_MAX_BOOL (SelectMaxSRing<bool,T>) 191-210,
 *   BOOL_COPY1ST 96-141, BOOL_COPY2ND 50-94 (add() throws there; here it is an error code).
 * A NULL value pointer means a pattern (bool) matrix whose stored values are all "true".
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>
#include <limits.h>

enum { SR_PLUS_TIMES = 0, SR_MIN_PLUS = 1, SR_SELECT2ND = 2, SR_SELECT_MAX = 3,
       SR_SELECT_MAX_BOOL = 4, SR_BOOL_COPY1ST = 5, SR_BOOL_COPY2ND = 6 };
enum { DT_BOOL = 0, DT_I32 = 1, DT_I64 = 2, DT_F32 = 3, DT_F64 = 4 };
enum { ORC_OK = 0, ORC_EDIM = 3002, ORC_ENOMEM = 10, ORC_EUNSUP = 11, ORC_EADD = 13 };

typedef struct {
  int64_t nrow, ncol, nnz;
  const int64_t* cp;   /* ncol+1 */
  const int32_t* ir;   /* nnz, ascending within a column */
  const void* val;     /* nnz of dtype, or NULL (pattern) */
} orc_csc;

static int64_t pow2_at_least(int64_t x, int64_t lo) {
  int64_t s = lo;
  while (s < x) s <<= 1;
  return s;
}

/* estimateFLOP: flop[j] = sum_{k in B(:,j)} nnz(A(:,k)) */
int orc_flops(const orc_csc* A, const orc_csc* B, int64_t* flop_per_col, int64_t* total) {
  if (A->ncol != B->nrow) return ORC_EDIM;
  int64_t t = 0;
#pragma omp parallel for schedule(dynamic, 256) reduction(+ : t)
  for (int64_t j = 0; j < B->ncol; ++j) {
    int64_t f = 0;
    for (int64_t p = B->cp[j]; p < B->cp[j + 1]; ++p) {
      int32_t k = B->ir[p];
      f += A->cp[k + 1] - A->cp[k];
    }
    if (flop_per_col) flop_per_col[j] = f;
    t += f;
  }
  if (total) *total = t;
  return ORC_OK;
}

/* estimateNNZ_Hash: distinct rows per output column (keys-only hash) */
int orc_symbolic(const orc_csc* A, const orc_csc* B, int64_t* nnz_per_col, int64_t* total) {
  if (A->ncol != B->nrow) return ORC_EDIM;
  int64_t t = 0;
  int bad = 0;
#pragma omp parallel reduction(+ : t) reduction(| : bad)
  {
    int64_t cap = 0;
    int32_t* tab = NULL;
#pragma omp for schedule(dynamic, 64)
    for (int64_t j = 0; j < B->ncol; ++j) {
      int64_t f = 0;
      for (int64_t p = B->cp[j]; p < B->cp[j + 1]; ++p) f += A->cp[B->ir[p] + 1] - A->cp[B->ir[p]];
      int64_t n = 0;
      if (f > 0) {
        int64_t hs = pow2_at_least(f, 16);
        if (hs > cap) { free(tab); cap = hs; tab = (int32_t*)malloc(sizeof(int32_t) * cap); if (!tab) { bad = 1; cap = 0; continue; } }
        for (int64_t s = 0; s < hs; ++s) tab[s] = -1;
        for (int64_t p = B->cp[j]; p < B->cp[j + 1]; ++p) {
          int32_t k = B->ir[p];
          for (int64_t q = A->cp[k]; q < A->cp[k + 1]; ++q) {
            int32_t key = A->ir[q];
            int64_t h = ((int64_t)key * 107) & (hs - 1);
            for (;;) {
              if (tab[h] == key) break;
              if (tab[h] == -1) { tab[h] = key; ++n; break; }
              h = (h + 1) & (hs - 1);
            }
          }
        }
      }
      if (nnz_per_col) nnz_per_col[j] = n;
      t += n;
    }
    free(tab);
  }
  if (total) *total = t;
  return bad ? ORC_ENOMEM : ORC_OK;
}

/* ---- semiring scalar ops per value type, generated by macro ---------------------- */
#define ORC_MAXV_double DBL_MAX
#define ORC_MAXV_float FLT_MAX
#define ORC_MAXV_int64_t INT64_MAX
#define ORC_MAXV_int32_t INT32_MAX
#define ORC_MAXV_uint8_t 1

/* one hash-table slot */
#define DEFINE_ORACLE(T, SUF)                                                              \
  typedef struct { int32_t key; int32_t pos; T val; } slot_##SUF;                          \
  static int cmp_slot_##SUF(const void* a, const void* b) {                                \
    int32_t x = ((const slot_##SUF*)a)->key, y = ((const slot_##SUF*)b)->key;              \
    return (x > y) - (x < y);                                                              \
  }                                                                                        \
  static int cmp_slot_pos_##SUF(const void* a, const void* b) {                            \
    const slot_##SUF *x = (const slot_##SUF*)a, *y = (const slot_##SUF*)b;                 \
    if (x->key != y->key) return (x->key > y->key) - (x->key < y->key);                    \
    return (x->pos > y->pos) - (x->pos < y->pos);                                          \
  }                                                                                        \
  static T av_##SUF(const void* v, int64_t i) { return v ? ((const T*)v)[i] : (T)1; }      \
  static T mul_##SUF(int sr, T a, T b) {                                                   \
    switch (sr) {                                                                          \
      case SR_PLUS_TIMES: case SR_SELECT_MAX: return (T)(a * b);                           \
      case SR_MIN_PLUS: {                                                                  \
        const T inf = (T)ORC_MAXV_##T;                                                     \
        if (a == inf || b == inf) return inf;                                              \
        return (T)(a + b);                                                                 \
      }                                                                                    \
      case SR_SELECT2ND: case SR_SELECT_MAX_BOOL: case SR_BOOL_COPY2ND: return b;          \
      case SR_BOOL_COPY1ST: return a;                                                      \
    }                                                                                      \
    return b;                                                                              \
  }                                                                                        \
  /* add(arg1 = new product, arg2 = existing) exactly as mtSpGEMM.h:583 calls it */        \
  static T add_##SUF(int sr, T newp, T existing, int* err) {                               \
    switch (sr) {                                                                          \
      case SR_PLUS_TIMES: return (T)(newp + existing);                                     \
      case SR_MIN_PLUS: return newp < existing ? newp : existing;                          \
      case SR_SELECT2ND: return existing;                                                  \
      case SR_SELECT_MAX: case SR_SELECT_MAX_BOOL: return newp > existing ? newp : existing; \
      default: *err = 1; return existing;                                                  \
    }                                                                                      \
  }                                                                                        \
  static int spgemm_##SUF(int sr, const orc_csc* A, const orc_csc* B, int sort,            \
                          int64_t* cp_out, int32_t* ir_out, T* val_out, int64_t nnz_cap) { \
    int bad = 0, adderr = 0;                                                               \
    (void)nnz_cap;                                                                         \
    _Pragma("omp parallel reduction(| : bad, adderr)")                                     \
    {                                                                                      \
      int64_t cap = 0;                                                                     \
      slot_##SUF* tab = NULL;                                                              \
      _Pragma("omp for schedule(dynamic, 64)")                                             \
      for (int64_t j = 0; j < B->ncol; ++j) {                                              \
        int64_t nz = cp_out[j + 1] - cp_out[j];                                            \
        if (nz == 0) continue;                                                             \
        int64_t hs = pow2_at_least(nz, 16);                                                \
        if (hs > cap) {                                                                    \
          free(tab); cap = hs; tab = (slot_##SUF*)malloc(sizeof(slot_##SUF) * cap);        \
          if (!tab) { bad = 1; cap = 0; continue; }                                        \
        }                                                                                  \
        for (int64_t s = 0; s < hs; ++s) tab[s].key = -1;                                  \
        for (int64_t p = B->cp[j]; p < B->cp[j + 1]; ++p) {                                \
          int32_t k = B->ir[p];                                                            \
          T bv = av_##SUF(B->val, p);                                                      \
          for (int64_t q = A->cp[k]; q < A->cp[k + 1]; ++q) {                              \
            T m = mul_##SUF(sr, av_##SUF(A->val, q), bv);                                  \
            int32_t key = A->ir[q];                                                        \
            int64_t h = ((int64_t)key * 107) & (hs - 1);                                   \
            for (;;) {                                                                     \
              if (tab[h].key == key) { int e = 0; tab[h].val = add_##SUF(sr, m, tab[h].val, &e); adderr |= e; break; } \
              if (tab[h].key == -1) { tab[h].key = key; tab[h].val = m; break; }           \
              h = (h + 1) & (hs - 1);                                                      \
            }                                                                              \
          }                                                                                \
        }                                                                                  \
        int64_t n = 0;                                                                     \
        for (int64_t s = 0; s < hs; ++s) if (tab[s].key != -1) tab[n++] = tab[s];          \
        if (n != nz) { bad = 1; continue; }                                                \
        if (sort) qsort(tab, (size_t)n, sizeof(slot_##SUF), cmp_slot_##SUF);               \
        for (int64_t e = 0; e < n; ++e) {                                                  \
          ir_out[cp_out[j] + e] = tab[e].key;                                              \
          if (val_out) val_out[cp_out[j] + e] = tab[e].val;                                \
        }                                                                                  \
      }                                                                                    \
      free(tab);                                                                           \
    }                                                                                      \
    if (adderr) return ORC_EADD;                                                           \
    return bad ? ORC_ENOMEM : ORC_OK;                                                      \
  }                                                                                        \
  /* Multi-list merge in MultiwayMergeHash order (SerialMergeHash, MultiwayMerge.h:320-405):  */ \
  /* lists are column-sorted CSCs of equal shape; duplicates combined in list order,           */ \
  /* acc = add(next, acc) = SR::add(curval, existing) (:357): for Select2nd the first list     */ \
  /* wins.  The heap MultiwayMerge (SerialMerge, :184-231) calls SR::add(existing, new) in     */ \
  /* heap-pop order instead, which differs for Select2nd only; tests/golden/merge.npz holds    */ \
  /* both reference outputs, and this order is the one equal to the 1-rank product (min-k).    */ \
  static int merge_##SUF(int sr, int nl, const orc_csc* L, int64_t* cp_out, int32_t* ir_out, \
                         T* val_out, int count_only) {                                     \
    int64_t ncol = L[0].ncol, nrow = L[0].nrow;                                            \
    int adderr = 0, bad = 0;                                                               \
    _Pragma("omp parallel reduction(| : adderr, bad)")                                     \
    {                                                                                      \
      int64_t cap = 0;                                                                     \
      slot_##SUF* buf = NULL;                                                              \
      _Pragma("omp for schedule(dynamic, 64)")                                             \
      for (int64_t j = 0; j < ncol; ++j) {                                                 \
        int64_t tot = 0;                                                                   \
        for (int l = 0; l < nl; ++l) tot += L[l].cp[j + 1] - L[l].cp[j];                   \
        if (tot > cap) { free(buf); cap = tot; buf = (slot_##SUF*)malloc(sizeof(slot_##SUF) * cap); if (!buf) { bad = 1; cap = 0; continue; } } \
        int64_t n = 0;                                                                     \
        for (int l = 0; l < nl; ++l)                                                       \
          for (int64_t p = L[l].cp[j]; p < L[l].cp[j + 1]; ++p) {                          \
            buf[n].key = L[l].ir[p]; buf[n].pos = (int32_t)n;                              \
            buf[n].val = av_##SUF(L[l].val, p); ++n;                                       \
          }                                                                                \
        /* stable by (row, list order): ties broken by insertion position */              \
        qsort(buf, (size_t)n, sizeof(slot_##SUF), cmp_slot_pos_##SUF);                    \
        int64_t m = 0;                                                                     \
        for (int64_t a = 0; a < n; ++a) {                                                  \
          if (m > 0 && buf[m - 1].key == buf[a].key) {                                     \
            int e = 0; buf[m - 1].val = add_##SUF(sr, buf[a].val, buf[m - 1].val, &e); adderr |= e; \
          } else buf[m++] = buf[a];                                                        \
        }                                                                                  \
        if (count_only) { cp_out[j] = m; continue; }                                       \
        for (int64_t a = 0; a < m; ++a) {                                                  \
          ir_out[cp_out[j] + a] = buf[a].key;                                              \
          if (val_out) val_out[cp_out[j] + a] = buf[a].val;                                \
        }                                                                                  \
      }                                                                                    \
      free(buf);                                                                           \
    }                                                                                      \
    (void)nrow;                                                                            \
    if (adderr) return ORC_EADD;                                                           \
    return bad ? ORC_ENOMEM : ORC_OK;                                                      \
  }

DEFINE_ORACLE(double, f64)
DEFINE_ORACLE(float, f32)
DEFINE_ORACLE(int64_t, i64)
DEFINE_ORACLE(int32_t, i32)

/* bool: PlusTimes<bool,bool> is OR-AND; all bool semirings reduce to "some product" */
typedef struct { int32_t key; int32_t pos; uint8_t val; } slot_b8;

static size_t dt_size(int dt) {
  switch (dt) { case DT_BOOL: return 1; case DT_I32: case DT_F32: return 4; default: return 8; }
}

/*
 * Full product.  Caller passes cp_out (ncol(B)+1) and gets malloc'd ir/val (free with
 * orc_free).  Values are computed in dtype `dt` (A and B values are of that type, or NULL).
 */
int orc_spgemm(int sr, int dt, const orc_csc* A, const orc_csc* B, int sort, int64_t* flops,
               int64_t* cp_out, int32_t** ir_out, void** val_out, int64_t* nnz_out) {
  if (A->ncol != B->nrow) return ORC_EDIM;
  if (flops) orc_flops(A, B, NULL, flops);
  int64_t* cnt = (int64_t*)malloc(sizeof(int64_t) * (size_t)(B->ncol > 0 ? B->ncol : 1));
  if (!cnt) return ORC_ENOMEM;
  int64_t tot = 0;
  int rc = orc_symbolic(A, B, cnt, &tot);
  if (rc) { free(cnt); return rc; }
  cp_out[0] = 0;
  for (int64_t j = 0; j < B->ncol; ++j) cp_out[j + 1] = cp_out[j] + cnt[j];
  free(cnt);
  *nnz_out = tot;
  *ir_out = (int32_t*)malloc(sizeof(int32_t) * (size_t)(tot > 0 ? tot : 1));
  *val_out = malloc(dt_size(dt) * (size_t)(tot > 0 ? tot : 1));
  if (!*ir_out || !*val_out) return ORC_ENOMEM;
  switch (dt) {
    case DT_F64: return spgemm_f64(sr, A, B, sort, cp_out, *ir_out, (double*)*val_out, tot);
    case DT_F32: return spgemm_f32(sr, A, B, sort, cp_out, *ir_out, (float*)*val_out, tot);
    case DT_I64: return spgemm_i64(sr, A, B, sort, cp_out, *ir_out, (int64_t*)*val_out, tot);
    case DT_I32: return spgemm_i32(sr, A, B, sort, cp_out, *ir_out, (int32_t*)*val_out, tot);
    case DT_BOOL: {
      /* compute in i32 (0/1 values) and narrow: OR-AND / select semantics coincide */
      int32_t* tmp = (int32_t*)malloc(sizeof(int32_t) * (size_t)(tot > 0 ? tot : 1));
      if (!tmp) return ORC_ENOMEM;
      orc_csc A2 = *A, B2 = *B;
      int32_t *av = NULL, *bv = NULL;
      if (A->val) { av = (int32_t*)malloc(4 * (size_t)(A->nnz + 1)); for (int64_t i = 0; i < A->nnz; ++i) av[i] = ((const uint8_t*)A->val)[i] != 0; A2.val = av; }
      if (B->val) { bv = (int32_t*)malloc(4 * (size_t)(B->nnz + 1)); for (int64_t i = 0; i < B->nnz; ++i) bv[i] = ((const uint8_t*)B->val)[i] != 0; B2.val = bv; }
      int r = spgemm_i32(sr == SR_PLUS_TIMES ? SR_SELECT_MAX : sr, &A2, &B2, sort, cp_out, *ir_out, tmp, tot);
      for (int64_t i = 0; i < tot; ++i) ((uint8_t*)*val_out)[i] = tmp[i] != 0;
      free(tmp); free(av); free(bv);
      return r;
    }
  }
  return ORC_EUNSUP;
}

/* Two-call merge: first with ir_out == NULL fills cp_out with the merged colptr. */
int orc_merge(int sr, int dt, int nlists, const orc_csc* lists, int64_t* cp_out, int32_t** ir_out,
              void** val_out, int64_t* nnz_out) {
  if (nlists <= 0) return ORC_EDIM;
  for (int l = 1; l < nlists; ++l)
    if (lists[l].ncol != lists[0].ncol || lists[l].nrow != lists[0].nrow) return ORC_EDIM;
  int64_t ncol = lists[0].ncol;
  int64_t* cnt = (int64_t*)malloc(sizeof(int64_t) * (size_t)(ncol + 1));
  if (!cnt) return ORC_ENOMEM;
  int rc;
  switch (dt) {
    case DT_F64: rc = merge_f64(sr, nlists, lists, cnt, NULL, NULL, 1); break;
    case DT_F32: rc = merge_f32(sr, nlists, lists, cnt, NULL, NULL, 1); break;
    case DT_I64: rc = merge_i64(sr, nlists, lists, cnt, NULL, NULL, 1); break;
    case DT_I32: rc = merge_i32(sr, nlists, lists, cnt, NULL, NULL, 1); break;
    default: free(cnt); return ORC_EUNSUP;
  }
  if (rc) { free(cnt); return rc; }
  cp_out[0] = 0;
  for (int64_t j = 0; j < ncol; ++j) cp_out[j + 1] = cp_out[j] + cnt[j];
  free(cnt);
  int64_t tot = cp_out[ncol];
  *nnz_out = tot;
  *ir_out = (int32_t*)malloc(sizeof(int32_t) * (size_t)(tot > 0 ? tot : 1));
  *val_out = malloc(dt_size(dt) * (size_t)(tot > 0 ? tot : 1));
  if (!*ir_out || !*val_out) return ORC_ENOMEM;
  switch (dt) {
    case DT_F64: return merge_f64(sr, nlists, lists, cp_out, *ir_out, (double*)*val_out, 0);
    case DT_F32: return merge_f32(sr, nlists, lists, cp_out, *ir_out, (float*)*val_out, 0);
    case DT_I64: return merge_i64(sr, nlists, lists, cp_out, *ir_out, (int64_t*)*val_out, 0);
    case DT_I32: return merge_i32(sr, nlists, lists, cp_out, *ir_out, (int32_t*)*val_out, 0);
  }
  return ORC_EUNSUP;
}

void orc_free(void* p) { free(p); }

/* ------------------------------------------------------------------ MCLPruneRecoverySelect */
static int cmp_desc(const void* a, const void* b) {
  const double x = *(const double*)a, y = *(const double*)b;
  return (x < y) - (x > y);
}

/* Kselect1 on one column (SpParMat.cpp:1536-1548 partial_sort greater<>, :1660-1668 pick) */
static double kth_largest(const double* v, int64_t n, int64_t k, double* scratch) {
  if (n == 0) return DBL_MIN;
  memcpy(scratch, v, sizeof(double) * (size_t)n);
  qsort(scratch, (size_t)n, sizeof(double), cmp_desc);
  return n >= k ? scratch[k - 1] : scratch[n - 1];
}

/* in: f64 CSC (column-complete).  out arrays: cp_out[ncol+1]; ir_out, val_out malloc'd.
   stats[0..2] = recovered, selected, recovered after selection. */
int orc_mcl_prune(const orc_csc* A, double thr, int64_t S, int64_t R, double pct, int64_t* cp_out,
                  int32_t** ir_out, double** val_out, int64_t* stats) {
  const double* val = (const double*)A->val;
  double* th = (double*)malloc(sizeof(double) * (size_t)(A->ncol + 1));
  double* scratch = (double*)malloc(sizeof(double) * (size_t)(A->nnz + 1));
  if (!th || !scratch) { free(th); free(scratch); return ORC_ENOMEM; }
  stats[0] = stats[1] = stats[2] = 0;
  for (int64_t j = 0; j < A->ncol; ++j) {
    const int64_t a = A->cp[j], b = A->cp[j + 1], nu = b - a;
    int64_t np = 0;
    double sp = 0.0;
    for (int64_t k = a; k < b; ++k)
      if (!(val[k] <= thr)) { ++np; sp += val[k]; }   /* Prune(bind2nd(less_equal, thr)) keeps v > thr */
    th[j] = thr;
    if (np < R && nu > np && sp < pct) {              /* ParFriends.h:207-233 */
      th[j] = kth_largest(val + a, nu, R, scratch);
      stats[0]++;
    } else if (S > 0 && np > S) {                     /* ParFriends.h:251-267 */
      const double t = kth_largest(val + a, nu, S, scratch);
      th[j] = t;
      stats[1]++;
      if (R > 0) {                                    /* ParFriends.h:290-333 */
        int64_t n1 = 0;
        double s1 = 0.0;
        for (int64_t k = a; k < b; ++k)
          if (!(val[k] < t)) { ++n1; s1 += val[k]; }
        if (n1 < R && s1 < pct) { th[j] = kth_largest(val + a, nu, R, scratch); stats[2]++; }
      }
    }
  }
  cp_out[0] = 0;
  for (int64_t j = 0; j < A->ncol; ++j) {
    int64_t c = 0;
    for (int64_t k = A->cp[j]; k < A->cp[j + 1]; ++k) c += !(val[k] < th[j]);
    cp_out[j + 1] = cp_out[j] + c;
  }
  const int64_t nnz = cp_out[A->ncol];
  int32_t* ir = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nnz + 1));
  double* v = (double*)malloc(sizeof(double) * (size_t)(nnz + 1));
  if (!ir || !v) { free(ir); free(v); free(th); free(scratch); return ORC_ENOMEM; }
  int64_t o = 0;
  for (int64_t j = 0; j < A->ncol; ++j)
    for (int64_t k = A->cp[j]; k < A->cp[j + 1]; ++k)
      if (!(val[k] < th[j])) { ir[o] = A->ir[k]; v[o] = val[k]; ++o; }
  *ir_out = ir;
  *val_out = v;
  free(th);
  free(scratch);
  return ORC_OK;
}
