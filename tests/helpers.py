"""Shared test utilities: fixture loading, the oracle binding (tests only), comparisons."""
import ctypes
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")

SR = {"plus_times": 0, "min_plus": 1, "select2nd": 2, "select_max": 3,
      "select_max_bool": 4, "bool_copy1st": 5, "bool_copy2nd": 6}
DT = {"bool": 0, "i32": 1, "i64": 2, "f32": 3, "f64": 4}
NP_DT = {0: np.uint8, 1: np.int32, 2: np.int64, 3: np.float32, 4: np.float64}

# fixture tag prefix -> (semiring, dtype, A is pattern)
TAGS = {"pt_f64": ("plus_times", "f64", False), "mp_f64": ("min_plus", "f64", False),
        "pt_i64": ("plus_times", "i64", False), "mp_i64": ("min_plus", "i64", False),
        "s2_i64": ("select2nd", "i64", False), "sm_i64": ("select_max", "i64", False),
        "smb_i64": ("select_max_bool", "i64", True)}


class Csc:
    """Host CSC: int64 colptr, int32 rows, values (or None = pattern)."""

    def __init__(self, nrow, ncol, cp, ir, val):
        self.nrow, self.ncol = int(nrow), int(ncol)
        self.cp = np.ascontiguousarray(cp, np.int64)
        self.ir = np.ascontiguousarray(ir, np.int32)
        self.val = None if val is None else np.ascontiguousarray(val)

    @property
    def nnz(self):
        return int(self.cp[-1])

    def to_scipy(self):
        import scipy.sparse as sp
        v = np.ones(self.nnz) if self.val is None else self.val
        return sp.csc_matrix((v, self.ir, self.cp), shape=(self.nrow, self.ncol))


def load_fixture(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


def fixture_inputs(z, tag):
    """(A, B) host CSCs for a fixture product tag, with values converted for its dtype."""
    sr, dt, a_pattern = TAGS[tag.rsplit("_", 1)[0]]
    ash = z["A_shape"]
    aval = z["A_ival"] if dt == "i64" else z["A_val"]
    A = Csc(ash[0], ash[1], z["A_cp"], z["A_ir"], None if a_pattern else aval.astype(NP_DT[DT[dt]]))
    if "B_cp" in z.files:
        bsh = z["B_shape"]
        B = Csc(bsh[0], bsh[1], z["B_cp"], z["B_ir"], z["B_val"].astype(NP_DT[DT[dt]]))
    else:
        B = Csc(ash[0], ash[1], z["A_cp"], z["A_ir"], aval.astype(NP_DT[DT[dt]]))
    return A, B, sr, dt


def fixture_product(z, tag):
    cp = z[f"C_{tag}_cp"]
    return Csc(0, len(cp) - 1, cp, z[f"C_{tag}_ir"], z[f"C_{tag}_val"])


def canonical_sha256(cp, ir, val):
    import sys
    sys.path.insert(0, GOLDEN)
    from cbm import canonical_sha256 as f
    return f(cp, ir, val)


# ---------------------------------------------------------------------------------- oracle
_CT = {np.dtype(np.uint8): ctypes.c_uint8, np.dtype(np.int32): ctypes.c_int32, np.dtype(np.int64): ctypes.c_int64,
       np.dtype(np.float32): ctypes.c_float, np.dtype(np.float64): ctypes.c_double}


def _copy_out(ptr, n, dtype):
    """n elements of `dtype` at a C pointer, copied (no 2/4 GiB limit, unlike ctypes.string_at)."""
    dtype = np.dtype(dtype)
    if n == 0:
        return np.zeros(0, dtype)
    return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(_CT[dtype])), (n,)).copy()


class _OrcCsc(ctypes.Structure):
    _fields_ = [("nrow", ctypes.c_int64), ("ncol", ctypes.c_int64), ("nnz", ctypes.c_int64),
                ("cp", ctypes.c_void_p), ("ir", ctypes.c_void_p), ("val", ctypes.c_void_p)]


_orc = None


def oracle_lib():
    """TEST INFRASTRUCTURE: the CPU restatement in oracle/oracle.c (parity checker only)."""
    global _orc
    if _orc is None:
        path = os.path.join(REPO, "oracle", "liboracle.so")
        if not os.path.exists(path):
            import subprocess
            subprocess.run(["make", "-C", os.path.join(REPO, "oracle")], check=True,
                           capture_output=True)
        _orc = ctypes.CDLL(path)
        _orc.orc_free.argtypes = [ctypes.c_void_p]
    return _orc


def _orc_view(M, keep):
    keep.append(M)
    return _OrcCsc(M.nrow, M.ncol, M.nnz, M.cp.ctypes.data, M.ir.ctypes.data,
                   None if M.val is None else M.val.ctypes.data)


def oracle_spgemm(A, B, sr, dt, sort=True):
    """Returns (C, multiplies, status)."""
    lib = oracle_lib()
    keep = []
    va, vb = _orc_view(A, keep), _orc_view(B, keep)
    cp = np.zeros(B.ncol + 1, np.int64)
    ir_p, val_p = ctypes.c_void_p(), ctypes.c_void_p()
    fl, nnz = ctypes.c_int64(0), ctypes.c_int64(0)
    rc = lib.orc_spgemm(SR[sr], DT[dt], ctypes.byref(va), ctypes.byref(vb), int(sort),
                        ctypes.byref(fl), cp.ctypes.data_as(ctypes.c_void_p),
                        ctypes.byref(ir_p), ctypes.byref(val_p), ctypes.byref(nnz))
    if rc != 0:
        for p in (ir_p, val_p):
            if p.value:
                lib.orc_free(p)
        return None, fl.value, rc
    n = nnz.value
    dtype = NP_DT[DT[dt]]
    ir = _copy_out(ir_p, n, np.int32)
    val = _copy_out(val_p, n, dtype)
    lib.orc_free(ir_p)
    lib.orc_free(val_p)
    return Csc(A.nrow, B.ncol, cp, ir, val), fl.value, 0


def oracle_merge(parts, sr, dt):
    lib = oracle_lib()
    keep = []
    arr = (_OrcCsc * len(parts))(*[_orc_view(P, keep) for P in parts])
    ncol = parts[0].ncol
    cp = np.zeros(ncol + 1, np.int64)
    ir_p, val_p, nnz = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_int64(0)
    rc = lib.orc_merge(SR[sr], DT[dt], len(parts), arr, cp.ctypes.data_as(ctypes.c_void_p),
                       ctypes.byref(ir_p), ctypes.byref(val_p), ctypes.byref(nnz))
    if rc != 0:
        return None, rc
    n = nnz.value
    dtype = NP_DT[DT[dt]]
    ir = _copy_out(ir_p, n, np.int32)
    val = _copy_out(val_p, n, dtype)
    lib.orc_free(ir_p)
    lib.orc_free(val_p)
    return Csc(parts[0].nrow, ncol, cp, ir, val), 0


# ------------------------------------------------------------------------------ comparison
def abs_product_sums(A, B):
    """Sum |a*b| per output entry (the cancellation-safe scale for the 1e-12 rule)."""
    import scipy.sparse as sp
    Aa = abs(A.to_scipy()).astype(np.float64)
    Ba = abs(B.to_scipy()).astype(np.float64)
    return sp.csc_matrix(Aa @ Ba)


def assert_same_product(C, R, dt, scale=None, rtol=1e-12, what=""):
    """Structure exact; values bit-exact for integer/bool dtypes, rtol-relative for floats
    (|c - r| <= rtol * max(|r|, sum|a*b|)), SURVEY §8a."""
    assert C.ncol == R.ncol, f"{what}: ncol {C.ncol} != {R.ncol}"
    assert np.array_equal(C.cp, R.cp), f"{what}: colptr differs (nnz {C.nnz} vs {R.nnz})"
    assert np.array_equal(C.ir, R.ir), f"{what}: row indices differ"
    if dt in ("f64", "f32"):
        c = C.val.astype(np.float64)
        r = R.val.astype(np.float64)
        s = np.abs(r)
        if scale is not None:
            s = np.maximum(s, scale)
        tol = rtol * s
        bad = np.abs(c - r) > tol
        bad &= ~(np.isinf(c) & np.isinf(r) & (np.sign(c) == np.sign(r)))
        assert not bad.any(), (f"{what}: {int(bad.sum())} values off, worst "
                               f"{float(np.max(np.abs(c - r)[bad]))}")
    else:
        assert np.array_equal(C.val.astype(np.int64), R.val.astype(np.int64)), f"{what}: values differ"


def sorted_dedup_ok(C):
    for j in range(C.ncol):
        seg = C.ir[C.cp[j]:C.cp[j + 1]]
        if len(seg) > 1 and not np.all(seg[1:] > seg[:-1]):
            return False
    return True


def oracle_mcl_prune(A, thr, select, recover, pct):
    """orc_mcl_prune (MCLPruneRecoverySelect restated): returns (Csc, (recovered, selected, rec2))."""
    lib = oracle_lib()
    keep = []
    va = _orc_view(A, keep)
    cp = np.zeros(A.ncol + 1, np.int64)
    ir_p, val_p = ctypes.c_void_p(), ctypes.c_void_p()
    st = np.zeros(3, np.int64)
    lib.orc_mcl_prune.argtypes = [ctypes.c_void_p, ctypes.c_double, ctypes.c_int64, ctypes.c_int64,
                                  ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.c_void_p]
    rc = lib.orc_mcl_prune(ctypes.byref(va), thr, select, recover, pct, cp.ctypes.data,
                           ctypes.byref(ir_p), ctypes.byref(val_p), st.ctypes.data)
    assert rc == 0
    n = int(cp[-1])
    ir = _copy_out(ir_p, n, np.int32)
    val = _copy_out(val_p, n, np.float64)
    lib.orc_free(ir_p)
    lib.orc_free(val_p)
    return Csc(A.nrow, A.ncol, cp, ir, val), tuple(int(x) for x in st)
