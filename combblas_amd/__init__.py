"""combblas_amd -- MI355X-native SpGEMM over semirings with CombBLAS's local-kernel interface.

Host-side mirror of the reference's local SpGEMM plugin point (include/CombBLAS/mtSpGEMM.h):

    LocalSpGEMMHash(SR, A, B, clearA=False, clearB=False, sort=True)   mtSpGEMM.h:465-470
    LocalHybridSpGEMM(SR, A, B, clearA=False, clearB=False, aux=None)   mtSpGEMM.h:212-217
    LocalSpGEMM(SR, A, B, clearA=False, clearB=False)                   mtSpGEMM.h:73-78
    EstimateLocalFLOP(SR, A, B)                                         mtSpGEMM.h:667-694
    MultiwayMerge(SR, lists, mdim, ndim, delarrs=False)                 MultiwayMerge.h:411-412

Semirings mirror include/CombBLAS/Semirings.h (PlusTimesSRing, MinPlusSRing, Select2ndSRing,
SelectMaxSRing, BoolCopy1stSRing, BoolCopy2ndSRing), parameterised by value dtype.  Matrices are
`SpDCCols` (device-resident CSC, the local matrix of SpDCCols.h:50) and products are `SpTuples`
(column-sorted triples, SpTuples.h:69) backed by a device CSC.  Every call goes through the C ABI
of libcbgpu.so (include/cbgpu.h); there is no CPU path in this package.
"""
import ctypes

import numpy as np

from . import _abi
from ._abi import CbgError

G500_SEED = 0xDECAFBAD   # the reference's default Graph500 user seed (RefGen21::init_random, RefGen21.h:306-318)

__all__ = ["Context", "SpDCCols", "SpTuples", "PlusTimesSRing", "MinPlusSRing", "Select2ndSRing",
           "SelectMaxSRing", "SelectMaxBoolSRing", "BoolCopy1stSRing", "BoolCopy2ndSRing",
           "LocalSpGEMMHash", "LocalHybridSpGEMM", "LocalSpGEMM", "EstimateLocalFLOP", "MultiwayMerge",
           "CbgError", "generate_rmat_host", "default_context", "G500_SEED", "RestrictionOp", "MIS2Restriction", "Transpose",
           "GalerkinRAP"]

_NP = {_abi.BOOL: np.uint8, _abi.I32: np.int32, _abi.I64: np.int64, _abi.F32: np.float32, _abi.F64: np.float64}
_DT = {"bool": _abi.BOOL, "i32": _abi.I32, "i64": _abi.I64, "f32": _abi.F32, "f64": _abi.F64,
       np.dtype(np.bool_): _abi.BOOL, np.dtype(np.uint8): _abi.BOOL, np.dtype(np.int32): _abi.I32,
       np.dtype(np.int64): _abi.I64, np.dtype(np.float32): _abi.F32, np.dtype(np.float64): _abi.F64}


def _dtype_code(d):
    if isinstance(d, int):
        return d
    if isinstance(d, str):
        return _DT[d]
    return _DT[np.dtype(d)]


# ------------------------------------------------------------------------------------ semirings
class _Semiring:
    code = None

    def __init__(self, dtype="f64"):
        self.dtype = _dtype_code(dtype)

    def __repr__(self):
        return f"{type(self).__name__}({self.dtype})"


class PlusTimesSRing(_Semiring):      # Semirings.h:212-233
    code = _abi.SR_PLUS_TIMES


class MinPlusSRing(_Semiring):        # Semirings.h:235-255 (inf_plus: max() is infinity)
    code = _abi.SR_MIN_PLUS


class Select2ndSRing(_Semiring):      # Semirings.h:143-163 (first contributor in B order wins)
    code = _abi.SR_SELECT2ND


class SelectMaxSRing(_Semiring):      # Semirings.h:165-190
    code = _abi.SR_SELECT_MAX


class SelectMaxBoolSRing(_Semiring):  # SelectMaxSRing<bool,T2>, Semirings.h:191-210 (A pattern)
    code = _abi.SR_SELECT_MAX_BOOL


class BoolCopy1stSRing(_Semiring):    # Semirings.h:96-141 (B pattern, add() is an error)
    code = _abi.SR_BOOL_COPY1ST


class BoolCopy2ndSRing(_Semiring):    # Semirings.h:50-94 (A pattern, add() is an error)
    code = _abi.SR_BOOL_COPY2ND


# -------------------------------------------------------------------------------------- context
class Context:
    """One HIP device + stream + workspace (cbg_ctx)."""

    def __init__(self, device=0):
        self._lib = _abi.lib()
        self._ptr = ctypes.c_void_p()
        _abi.check(self._lib.cbg_init(int(device), ctypes.byref(self._ptr)), "cbg_init")
        self.device = device

    def close(self):
        if self._ptr:
            self._lib.cbg_destroy(self._ptr)
            self._ptr = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def synchronize(self):
        _abi.check(self._lib.cbg_synchronize(self._ptr), "cbg_synchronize")

    def set_stream(self, hip_stream_ptr):
        _abi.check(self._lib.cbg_set_stream(self._ptr, ctypes.c_void_p(hip_stream_ptr)), "cbg_set_stream")

    def last_profile(self):
        p = _abi.Profile()
        _abi.check(self._lib.cbg_last_profile(self._ptr, ctypes.byref(p)), "cbg_last_profile")
        return {"flops_ms": p.flops_ms, "bin_ms": p.bin_ms, "symbolic_ms": p.symbolic_ms, "scan_ms": p.scan_ms,
                "numeric_ms": p.numeric_ms, "total_ms": p.total_ms, "multiplies": p.multiplies,
                "nnz_out": p.nnz_out, "bins": list(p.bins), "heavy_ms": p.heavy_ms, "known_items": p.known_items,
                "heavy_multiplies": p.heavy_multiplies, "heavy_nnz_b": p.heavy_nnz_b, "heavy_nnz_c": p.heavy_nnz_c}

    # raw ABI-level product (views in, device result out)
    def spgemm(self, A, B, sr, sort=True):
        res = _abi.CscResult()
        mults = ctypes.c_int64(0)
        va, vb = A._view(), B._view()
        st = self._lib.cbg_spgemm_local(self._ptr, ctypes.byref(va), ctypes.byref(vb), sr.code, sr.dtype,
                                        _abi.SORTED_COLS if sort else 0, ctypes.byref(res), ctypes.byref(mults))
        if st != _abi.OK:
            if res._owner:
                self._lib.cbg_result_free(self._ptr, ctypes.byref(res))
            raise CbgError(st, "cbg_spgemm_local")
        return SpDCCols._from_result(self, res)

    def merge(self, parts, sr, sort=True):
        arr = (_abi.CscResult * len(parts))(*[p._res for p in parts])
        res = _abi.CscResult()
        _abi.check(self._lib.cbg_merge(self._ptr, arr, len(parts), sr.code, sr.dtype,
                                       _abi.SORTED_COLS if sort else 0, ctypes.byref(res)), "cbg_merge")
        return SpDCCols._from_result(self, res)

    def generate_rmat(self, scale, edgefactor=16, seed=G500_SEED):
        """The reference's Graph500 Kronecker matrix (DistEdgeList::GenGraph500Data packed + SpParMat(DEL),
        DistEdgeList.cpp:223-280, SpParMat.cpp:3082-3196), built on this context's GPU."""
        res = _abi.CscResult()
        _abi.check(self._lib.cbg_generate_rmat(self._ptr, scale, edgefactor, seed, ctypes.byref(res)),
                   "cbg_generate_rmat")
        return SpDCCols._from_result(self, res)

    def rmat_block(self, scale, r0, r1, c0, c1, edgefactor=16, seed=G500_SEED):
        """Rows [r0, r1) x columns [c0, c1) of that matrix (local indices), built on the GPU."""
        res = _abi.CscResult()
        _abi.check(self._lib.cbg_rmat_block(self._ptr, scale, edgefactor, seed, r0, r1, c0, c1, ctypes.byref(res)),
                   "cbg_rmat_block")
        return SpDCCols._from_result(self, res)


_default = None


def default_context():
    global _default
    if _default is None:
        _default = Context(0)
    return _default


# -------------------------------------------------------------------------------------- matrices
class SpDCCols:
    """Device-resident local matrix (CSC, int64 colptr / int32 rows), owned by libcbgpu.

    Build from host arrays with SpDCCols.from_csc(ctx, nrow, ncol, colptr, rows, vals) or from a
    reference-style DCSC (cp, jc, ir, numx) with SpDCCols.from_dcsc(...)."""

    def __init__(self):
        self._ctx = None
        self._res = None
        self._keep = None

    @classmethod
    def _from_result(cls, ctx, res):
        m = cls()
        m._ctx, m._res = ctx, res
        return m

    @classmethod
    def from_csc(cls, ctx, nrow, ncol, colptr, rows, vals=None, dtype=None):
        cp = np.ascontiguousarray(colptr, np.int64)
        ir = np.ascontiguousarray(rows)
        if ir.dtype not in (np.int32, np.int64):
            ir = ir.astype(np.int64)
        v = None
        vt = _abi.BOOL
        if vals is not None:
            v = np.ascontiguousarray(vals if dtype is None else np.asarray(vals, dtype=_NP[_dtype_code(dtype)]))
            if v.dtype == np.bool_:
                v = v.astype(np.uint8)
            vt = _dtype_code(v.dtype)
        view = _abi.DcscView(int(nrow), int(ncol), int(cp[-1]), int(ncol), cp.ctypes.data, None, ir.ctypes.data,
                             ir.dtype.itemsize, 8, None if v is None else v.ctypes.data, vt, 0)
        res = _abi.CscResult()
        _abi.check(ctx._lib.cbg_upload(ctx._ptr, ctypes.byref(view), ctypes.byref(res)), "cbg_upload")
        return cls._from_result(ctx, res)

    def _view(self):
        v = _abi.DcscView()
        _abi.check(_abi.lib().cbg_result_view(ctypes.byref(self._res), ctypes.byref(v)), "cbg_result_view")
        return v

    def getnrow(self):
        return int(self._res.nrow)

    def getncol(self):
        return int(self._res.ncol)

    def getnnz(self):
        return int(self._res.nnz)

    @property
    def multiplies(self):
        return int(self._res.multiplies)

    @property
    def dtype(self):
        return _NP[self._res.val_type]

    def to_host(self):
        n, nc = self.getnnz(), self.getncol()
        cp = np.empty(nc + 1, np.int64)
        ir = np.empty(max(n, 1), np.int32)
        has_val = bool(self._res.val)
        val = np.empty(max(n, 1), self.dtype) if has_val else None
        _abi.check(self._ctx._lib.cbg_result_to_host(self._ctx._ptr, ctypes.byref(self._res), cp.ctypes.data,
                                                     ir.ctypes.data, None if val is None else val.ctypes.data),
                   "cbg_result_to_host")
        return cp, ir[:n], (None if val is None else val[:n])

    def select_columns(self, cols):
        """Columns `cols` (any order) as a new device matrix (cbg_col_select)."""
        c = np.ascontiguousarray(cols, np.int64)
        res = _abi.CscResult()
        _abi.check(self._ctx._lib.cbg_col_select(self._ctx._ptr, ctypes.byref(self._res), c.ctypes.data, len(c),
                                                 ctypes.byref(res)), "cbg_col_select")
        return SpDCCols._from_result(self._ctx, res)

    def fiber_codec(self, chunks=2):
        """The 3D fiber exchange's wire codec on this matrix as one outgoing partial (cbg_fiber_codec): the bytes its
        messages would put on the link and whether each chunk decodes back bit for bit."""
        st = _abi.CodecStats()
        _abi.check(self._ctx._lib.cbg_fiber_codec(self._ctx._ptr, ctypes.byref(self._res), int(chunks),
                                                  ctypes.byref(st)), "cbg_fiber_codec")
        return {k: getattr(st, k) for k, _ in _abi.CodecStats._fields_}

    def free(self):
        if self._res is not None and self._res._owner:
            self._ctx._lib.cbg_result_free(self._ctx._ptr, ctypes.byref(self._res))
        self._res = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class SpTuples(SpDCCols):
    """Column-sorted product triples (SpTuples.h:69) backed by the device CSC of the product."""

    def tuples(self):
        cp, ir, val = self.to_host()
        col = np.repeat(np.arange(self.getncol(), dtype=np.int64), np.diff(cp))
        return ir.astype(np.int64), col, val

    def rowindex(self):
        return self.tuples()[0]

    def colindex(self):
        return self.tuples()[1]

    def numvalue(self):
        return self.tuples()[2]


def _as_tuples(m):
    t = SpTuples._from_result(m._ctx, m._res)
    m._res = None
    return t


# ------------------------------------------------------------------------ reference entry points
def LocalSpGEMMHash(SR, A, B, clearA=False, clearB=False, sort=True):
    """mtSpGEMM.h:465-470.  clearA/clearB free the inputs after the call (ownership transfer)."""
    C = _as_tuples(A._ctx.spgemm(A, B, SR, sort=sort))
    if clearA:
        A.free()
    if clearB and B is not A:
        B.free()
    return C


def LocalHybridSpGEMM(SR, A, B, clearA=False, clearB=False, aux=None):
    """mtSpGEMM.h:212-217: always sorted; the heap/hash per-column switch is a CPU heuristic that the
    device kernel does not need (one hash/dense accumulator family covers both)."""
    return LocalSpGEMMHash(SR, A, B, clearA, clearB, sort=True)


def LocalSpGEMM(SR, A, B, clearA=False, clearB=False):
    """mtSpGEMM.h:73-78 (heap kernel in the reference; same product, min-k Select2nd rule)."""
    return LocalSpGEMMHash(SR, A, B, clearA, clearB, sort=True)


def EstimateLocalFLOP(SR, A, B, clearA=False, clearB=False):
    """mtSpGEMM.h:667-694: number of semiring multiplies of A*B."""
    ctx = A._ctx
    m, z = ctypes.c_int64(0), ctypes.c_int64(0)
    va, vb = A._view(), B._view()
    _abi.check(ctx._lib.cbg_estimate(ctx._ptr, ctypes.byref(va), ctypes.byref(vb), ctypes.byref(m),
                                     ctypes.byref(z)), "cbg_estimate")
    return int(m.value)


def EstimateLocalNNZ(A, B):
    """(multiplies, nnz(A*B)) from the symbolic pass alone (estimateFLOP + estimateNNZ_Hash, mtSpGEMM.h:810-938,
    1061-1139; exact on the device): no output is formed."""
    ctx = A._ctx
    m, z = ctypes.c_int64(0), ctypes.c_int64(0)
    va, vb = A._view(), B._view()
    _abi.check(ctx._lib.cbg_estimate(ctx._ptr, ctypes.byref(va), ctypes.byref(vb), ctypes.byref(m),
                                     ctypes.byref(z)), "cbg_estimate")
    return int(m.value), int(z.value)


def MultiwayMerge(SR, lists, mdim=0, ndim=0, delarrs=False):
    """MultiwayMerge.h:411-412: merge column-sorted partial products; duplicates -> SR::add."""
    if not lists:
        raise ValueError("MultiwayMerge needs at least one list")
    C = _as_tuples(lists[0]._ctx.merge(lists, SR))
    if delarrs:
        for L in lists:
            L.free()
    return C


def RestrictionOp(A, mt_seed=1, perm_seed=1383098845):
    """The reference's Galerkin restriction operator (3DSpGEMM/RestrictionOp.h:196-291) of the square matrix A
    on A's GPU, entry for entry: (R, RT) as device matrices, R (n x nagg) with R(i, agg(i)) = 1, RT = R^T.
    MIS2 on pattern(A) + pattern(A)^T without loops (:116-193, the MTRand stream of mt_seed), parents and
    Select2ndRandSR aggregation, aggregate columns permuted as RandPerm does (std::shuffle with
    std::default_random_engine(perm_seed)).  The defaults are the reference's DETERMINISTIC seeds."""
    ctx = A._ctx
    R, RT, nagg = _abi.CscResult(), _abi.CscResult(), ctypes.c_int64(0)
    _abi.check(ctx._lib.cbg_restriction_op(ctx._ptr, ctypes.byref(A._view()), int(mt_seed) & 0xFFFFFFFF,
                                           int(perm_seed) & 0xFFFFFFFF, ctypes.byref(R), ctypes.byref(RT),
                                           ctypes.byref(nagg)), "cbg_restriction_op")
    return SpDCCols._from_result(ctx, R), SpDCCols._from_result(ctx, RT)


def MIS2Restriction(G, seed=1):
    """A faster MIS-2 aggregation restriction of the graph of G (not the reference's R): Luby rounds with
    seeded distinct 64-bit priorities (no sequential random stream), every vertex joins the highest-priority
    set vertex within distance 1, else 2.  (R, RT) as device matrices.  G must be square and symmetric;
    self loops are ignored."""
    ctx = G._ctx
    R, RT, nagg = _abi.CscResult(), _abi.CscResult(), ctypes.c_int64(0)
    _abi.check(ctx._lib.cbg_mis2_restriction(ctx._ptr, ctypes.byref(G._view()), int(seed), ctypes.byref(R),
                                             ctypes.byref(RT), ctypes.byref(nagg)), "cbg_mis2_restriction")
    return SpDCCols._from_result(ctx, R), SpDCCols._from_result(ctx, RT)


def Transpose(A):
    """A^T as a new device matrix (SpDCCols::Transpose, SpDCCols.cpp:845); f64 values or a pattern."""
    ctx = A._ctx
    res = _abi.CscResult()
    _abi.check(ctx._lib.cbg_transpose(ctx._ptr, ctypes.byref(A._view()), ctypes.byref(res)), "cbg_transpose")
    return SpDCCols._from_result(ctx, res)


def GalerkinRAP(A, R, RT=None, fused=True):
    """C = R^T A R (RestrictionOp.cpp:188-196).  For an aggregation R (one nonzero per row) whose
    aggregates each gather at most 512 entries of A: one fused device pass (cbg_galerkin_rap,
    C.multiplies = nnz(A)).  Otherwise (or with fused=False) the reference's two products R^T A and
    (R^T A) R, with RT = R^T built on the device when not given."""
    ctx = A._ctx
    res = _abi.CscResult()
    st = _abi.EUNSUP
    if fused:
        st = ctx._lib.cbg_galerkin_rap(ctx._ptr, ctypes.byref(A._view()), ctypes.byref(R._view()),
                                       ctypes.byref(res))
    if st == _abi.EUNSUP:
        PT = PlusTimesSRing("f64")
        own = RT is None
        if own:
            RT = Transpose(R)
        RA = LocalSpGEMMHash(PT, RT, A)
        C = LocalSpGEMMHash(PT, RA, R)
        RA.free()
        if own:
            RT.free()
        return C
    _abi.check(st, "cbg_galerkin_rap")
    return SpDCCols._from_result(ctx, res)


def generate_rmat_host(scale, edgefactor=16, seed=G500_SEED):
    """The reference's Graph500 Kronecker matrix built on the host (no GPU needed): (n, colptr, rows, vals).
    `seed` is the Graph500 user seed (the reference's SEED environment variable, RefGen21.h:306-318)."""
    L = _abi.lib()
    h = _abi.HostCsc()
    _abi.check(L.cbg_rmat_host(scale, edgefactor, seed, ctypes.byref(h)), "cbg_rmat_host")
    try:
        n, nnz = h.ncol, h.nnz
        cp = np.ctypeslib.as_array(ctypes.cast(h.colptr, ctypes.POINTER(ctypes.c_int64)), (n + 1,)).copy()
        ir = np.ctypeslib.as_array(ctypes.cast(h.row, ctypes.POINTER(ctypes.c_int32)), (max(nnz, 1),))[:nnz].copy()
        val = np.ctypeslib.as_array(ctypes.cast(h.val, ctypes.POINTER(ctypes.c_double)), (max(nnz, 1),))[:nnz].copy()
    finally:
        L.cbg_host_free(ctypes.byref(h))
    return n, cp, ir, val


from .mcl import MCLPruneRecoverySelect, MemEfficientSpGEMM, MCL_DEFAULTS  # noqa: E402

__all__ += ["MCLPruneRecoverySelect", "MemEfficientSpGEMM", "MCL_DEFAULTS"]
