"""CBM1 binary matrix format (the refprobe exchange format) + canonical product hash.

  char magic[4]="CBM1"; int32 valtype (0=f64, 1=i64, 2=bool u8);
  int64 nrow, ncol, nnz; int64 colptr[ncol+1]; int64 row[nnz]; val[nnz]
"""
import hashlib

import numpy as np

_VT = {0: np.float64, 1: np.int64, 2: np.uint8}


def read_cbm(path):
    with open(path, "rb") as f:
        if f.read(4) != b"CBM1":
            raise ValueError(f"{path}: not a CBM1 file")
        vt = int(np.frombuffer(f.read(4), np.int32)[0])
        nrow, ncol, nnz = (int(x) for x in np.frombuffer(f.read(24), np.int64))
        cp = np.frombuffer(f.read(8 * (ncol + 1)), np.int64).copy()
        ir = np.frombuffer(f.read(8 * nnz), np.int64).copy()
        dt = _VT[vt]
        val = np.frombuffer(f.read(np.dtype(dt).itemsize * nnz), dt).copy()
    return {"vt": vt, "nrow": nrow, "ncol": ncol, "cp": cp, "ir": ir, "val": val}


def write_cbm(path, M):
    vt = int(M["vt"])
    with open(path, "wb") as f:
        f.write(b"CBM1")
        f.write(np.int32(vt).tobytes())
        nnz = len(M["ir"])
        f.write(np.array([M["nrow"], M["ncol"], nnz], np.int64).tobytes())
        f.write(np.asarray(M["cp"], np.int64).tobytes())
        f.write(np.asarray(M["ir"], np.int64).tobytes())
        f.write(np.asarray(M["val"], _VT[vt]).tobytes())


def canonical_sha256(cp, ir, val):
    """SHA-256 over (colptr int64 LE, rows int32 LE, values LE in their own dtype) of a
    column-sorted, duplicate-free CSC.  Same definition in tests and fixtures."""
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(cp, dtype="<i8").tobytes())
    h.update(np.ascontiguousarray(ir, dtype="<i4").tobytes())
    v = np.ascontiguousarray(val)
    if v.dtype == np.bool_:
        v = v.astype(np.uint8)
    h.update(v.astype(v.dtype.newbyteorder("<")).tobytes())
    return h.hexdigest()
