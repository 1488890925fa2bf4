"""ctypes declarations of include/cbgpu.h (the C ABI of libcbgpu.so).

The product path loads ONLY libcbgpu.so (built in-tree by `make -C combblas_amd/csrc`).  There is
no CPU fallback: if the library is missing, importing this module raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
_DEFAULT = os.path.join(_HERE, "libcbgpu.so")
LIB_PATH = os.environ.get("CBG_LIB_PATH") or _DEFAULT   # override: tuning variants

# cbg_status
OK, EDIM, EALIAS, ENOMEM, EUNSUP, EDEVICE, EADD, EINVAL, ECOMM = 0, 3002, 3005, 10, 11, 12, 13, 14, 15
# cbg_semiring
SR_PLUS_TIMES, SR_MIN_PLUS, SR_SELECT2ND, SR_SELECT_MAX, SR_SELECT_MAX_BOOL, SR_BOOL_COPY1ST, SR_BOOL_COPY2ND = range(7)
# cbg_dtype
BOOL, I32, I64, F32, F64 = range(5)
SORTED_COLS, KEEP_ON_DEVICE = 1, 2
# include/cbgpu.h CBG_ABI_VERSION these declarations follow: the library writes structs the caller allocates
# (cbg_profile, cbg_grid_stats), so a library of another ABI version is refused at load
ABI_VERSION = 4


class DcscView(ctypes.Structure):
    _fields_ = [("nrow", ctypes.c_int64), ("ncol", ctypes.c_int64), ("nnz", ctypes.c_int64),
                ("nzc", ctypes.c_int64), ("cp", ctypes.c_void_p), ("jc", ctypes.c_void_p),
                ("ir", ctypes.c_void_p), ("idx_bytes", ctypes.c_int32), ("ptr_bytes", ctypes.c_int32),
                ("val", ctypes.c_void_p), ("val_type", ctypes.c_int), ("on_device", ctypes.c_int32)]


class CscResult(ctypes.Structure):
    _fields_ = [("nrow", ctypes.c_int64), ("ncol", ctypes.c_int64), ("nnz", ctypes.c_int64),
                ("colptr", ctypes.c_void_p), ("row", ctypes.c_void_p), ("val", ctypes.c_void_p),
                ("val_type", ctypes.c_int), ("multiplies", ctypes.c_int64), ("_owner", ctypes.c_void_p)]


class Profile(ctypes.Structure):
    _fields_ = [("flops_ms", ctypes.c_double), ("bin_ms", ctypes.c_double), ("symbolic_ms", ctypes.c_double),
                ("scan_ms", ctypes.c_double), ("numeric_ms", ctypes.c_double), ("total_ms", ctypes.c_double),
                ("multiplies", ctypes.c_int64), ("nnz_out", ctypes.c_int64), ("bins", ctypes.c_int64 * 16),
                ("heavy_ms", ctypes.c_double), ("known_items", ctypes.c_int64),
                ("heavy_multiplies", ctypes.c_int64), ("heavy_nnz_b", ctypes.c_int64), ("heavy_nnz_c", ctypes.c_int64)]


class HostCsc(ctypes.Structure):
    _fields_ = [("nrow", ctypes.c_int64), ("ncol", ctypes.c_int64), ("nnz", ctypes.c_int64),
                ("colptr", ctypes.c_void_p), ("row", ctypes.c_void_p), ("val", ctypes.c_void_p)]


class MclStats(ctypes.Structure):
    _fields_ = [("recovered", ctypes.c_int64), ("selected", ctypes.c_int64),
                ("recovered_after_select", ctypes.c_int64), ("nnz_in", ctypes.c_int64), ("nnz_out", ctypes.c_int64)]


class GridStats(ctypes.Structure):
    _fields_ = [("multiplies", ctypes.c_int64), ("bcast_bytes", ctypes.c_int64), ("fiber_bytes", ctypes.c_int64),
                ("bcast_ms", ctypes.c_double), ("local_ms", ctypes.c_double), ("merge_ms", ctypes.c_double),
                ("fiber_ms", ctypes.c_double), ("total_ms", ctypes.c_double), ("stages", ctypes.c_int32),
                ("fiber_xfer_ms", ctypes.c_double),
                ("heavy_ms", ctypes.c_double), ("heavy_multiplies", ctypes.c_int64), ("heavy_nnz_b", ctypes.c_int64),
                ("heavy_nnz_c", ctypes.c_int64), ("local_nnz_out", ctypes.c_int64), ("local_nnz_b", ctypes.c_int64),
                ("local_ncol_b", ctypes.c_int64), ("local_products", ctypes.c_int32), ("fiber_mode", ctypes.c_int32)]


class CodecStats(ctypes.Structure):
    _fields_ = [("columns", ctypes.c_int64), ("entries", ctypes.c_int64), ("chunks", ctypes.c_int64),
                ("header_bytes", ctypes.c_int64), ("row_bytes", ctypes.c_int64), ("escape_bytes", ctypes.c_int64),
                ("value_bytes", ctypes.c_int64), ("value_header_bytes", ctypes.c_int64), ("wire_bytes", ctypes.c_int64),
                ("row_formats", ctypes.c_int32), ("value_formats", ctypes.c_int32), ("roundtrip_exact", ctypes.c_int32),
                ("mismatches", ctypes.c_int64), ("encode_ms", ctypes.c_double), ("decode_ms", ctypes.c_double)]


# cbg_transport callbacks (include/cbgpu.h)
BCAST_FN = ctypes.CFUNCTYPE(ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64,
                            ctypes.c_int32)
ALLTOALLV_FN = ctypes.CFUNCTYPE(ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                ctypes.POINTER(ctypes.c_int64), ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64))
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                ctypes.c_int64)


class Transport(ctypes.Structure):
    _fields_ = [("user", ctypes.c_void_p), ("bcast", BCAST_FN), ("alltoallv", ALLTOALLV_FN),
                ("allgather", ALLGATHER_FN), ("host_buffers", ctypes.c_int32)]


class GridInfo(ctypes.Structure):
    _fields_ = [("rccl", ctypes.c_int32), ("ranks", ctypes.c_int32 * 4)]


GROUP_ROW, GROUP_COL, GROUP_FIBER, GROUP_WORLD = range(4)
HALVES, RUNNING_MERGE = 4, 8

# name -> (restype, argtypes); must match include/cbgpu.h exactly
SIGNATURES = {
    "cbg_abi_version": (ctypes.c_int32, []),
    "cbg_strerror": (ctypes.c_char_p, [ctypes.c_int]),
    "cbg_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int32)]),
    "cbg_init": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "cbg_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "cbg_set_stream": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "cbg_synchronize": (ctypes.c_int, [ctypes.c_void_p]),
    "cbg_spgemm_local": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(DcscView), ctypes.POINTER(DcscView),
                                        ctypes.c_int, ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(CscResult),
                                        ctypes.POINTER(ctypes.c_int64)]),
    "cbg_estimate": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(DcscView), ctypes.POINTER(DcscView),
                                    ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
    "cbg_merge": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(CscResult), ctypes.c_int32, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(CscResult)]),
    "cbg_result_to_host": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(CscResult), ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_void_p]),
    "cbg_result_free": (None, [ctypes.c_void_p, ctypes.POINTER(CscResult)]),
    "cbg_upload": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(DcscView), ctypes.POINTER(CscResult)]),
    "cbg_result_view": (ctypes.c_int, [ctypes.POINTER(CscResult), ctypes.POINTER(DcscView)]),
    "cbg_last_profile": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Profile)]),
    "cbg_generate_rmat": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint64,
                                         ctypes.POINTER(CscResult)]),
    "cbg_rmat_block": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint64, ctypes.c_int64,
                                      ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.POINTER(CscResult)]),
    "cbg_mis2_restriction": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(DcscView), ctypes.c_uint64,
                                            ctypes.POINTER(CscResult), ctypes.POINTER(CscResult),
                                            ctypes.POINTER(ctypes.c_int64)]),
    "cbg_restriction_op": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(DcscView), ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.POINTER(CscResult), ctypes.POINTER(CscResult),
                                          ctypes.POINTER(ctypes.c_int64)]),
    "cbg_transpose": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(DcscView), ctypes.POINTER(CscResult)]),
    "cbg_galerkin_rap": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(DcscView), ctypes.POINTER(DcscView),
                                        ctypes.POINTER(CscResult)]),
    "cbg_rmat_host": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_uint64, ctypes.POINTER(HostCsc)]),
    "cbg_host_free": (None, [ctypes.POINTER(HostCsc)]),
    "cbg_mcl_prune": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(CscResult), ctypes.c_double, ctypes.c_int64,
                                     ctypes.c_int64, ctypes.c_double, ctypes.POINTER(CscResult),
                                     ctypes.POINTER(MclStats)]),
    "cbg_col_range": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(CscResult), ctypes.c_int64, ctypes.c_int64,
                                     ctypes.POINTER(CscResult)]),
    "cbg_col_concat": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(CscResult), ctypes.c_int32,
                                      ctypes.POINTER(CscResult)]),
    "cbg_col_select": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(CscResult), ctypes.c_void_p, ctypes.c_int64,
                                      ctypes.POINTER(CscResult)]),
    "cbg_rccl_unique_id": (ctypes.c_int, [ctypes.c_void_p]),
    "cbg_grid_create_rccl": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                                            ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                            ctypes.POINTER(ctypes.c_void_p)]),
    "cbg_grid_create": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Transport), ctypes.c_int32, ctypes.c_int32,
                                       ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(ctypes.c_void_p)]),
    "cbg_grid_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "cbg_grid_query": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(GridInfo)]),
    "cbg_spgemm_grid": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(DcscView), ctypes.POINTER(DcscView), ctypes.c_int,
                                       ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(CscResult),
                                       ctypes.POINTER(GridStats)]),
    "cbg_summa_layer": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(DcscView), ctypes.POINTER(DcscView), ctypes.c_int,
                                       ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(CscResult),
                                       ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(GridStats)]),
    "cbg_summa_estimate": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(DcscView), ctypes.POINTER(DcscView),
                                          ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
    "cbg_reduce_all": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(CscResult), ctypes.c_int32, ctypes.c_int,
                                      ctypes.c_int, ctypes.POINTER(CscResult), ctypes.POINTER(GridStats)]),
    "cbg_fiber_codec": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(CscResult), ctypes.c_int32,
                                       ctypes.POINTER(CodecStats)]),
}

_lib = None


def lib():
    """Load libcbgpu.so (raises OSError if it was not built: the product has no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OSError(f"{LIB_PATH} missing: build it with `make -C combblas_amd/csrc` "
                          "(or __graft_entry__.build()); there is no CPU fallback")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if LIB_PATH != _DEFAULT and not hasattr(L, name):
                continue   # an older tuning/diagnostic variant may lack newer entry points
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        v = L.cbg_abi_version() if hasattr(L, "cbg_abi_version") else None
        if v != ABI_VERSION:
            raise OSError(f"{LIB_PATH}: cbg_abi_version() = {v}, these bindings are ABI {ABI_VERSION}: rebuild it")
        _lib = L
    return _lib


class CbgError(RuntimeError):
    def __init__(self, status, where=""):
        self.status = status
        msg = lib().cbg_strerror(status).decode()
        super().__init__(f"{where}: cbgpu status {status} ({msg})" if where else f"cbgpu status {status} ({msg})")


def check(status, where=""):
    if status != OK:
        raise CbgError(status, where)
