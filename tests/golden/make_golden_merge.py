#!/usr/bin/env python3
"""Fixtures for the multi-list merge order (TEST INFRASTRUCTURE, build container only).

Runs the reference's own MultiwayMerge (heap, MultiwayMerge.h:411-526) and MultiwayMergeHash
(MultiwayMerge.h:536-684) through oracle/_ref/refprobe on k column-sorted partial products and stores
inputs + both outputs in tests/golden/merge.npz:

  * "split": the G500 s10 int64 matrix A, inner dimension cut into 4 contiguous parts,
    P_l = A[:, part_l] * A[part_l, :] under Select2nd (each made by the reference's LocalSpGEMMHash),
    merged in part order -- what a SUMMA / fiber merge sees.  The hash merge keeps SR::add(curval,
    existing) = the first list's value (:357), i.e. the global min-k rule of the 1-rank product.
  * "rand": 3 random lists with heavy overlap and list-distinct values, Select2nd and PlusTimes.

The heap merge combines duplicates with SR::add(existing, new) in heap-pop order (:213); for Select2nd
that keeps a later list's value, so the two reference merges differ there: the fixture records both.
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
PROBE = os.path.join(REPO, "oracle", "_ref", "refprobe")
sys.path.insert(0, HERE)
from cbm import read_cbm, write_cbm  # noqa: E402


def probe(*args):
    out = subprocess.run([PROBE, *args], check=True, capture_output=True, text=True).stdout
    lines = [l for l in out.splitlines() if l.startswith("{")]
    return json.loads(lines[-1]) if lines else {}


def csc_cols(M, c0, c1):
    cp = M["cp"][c0:c1 + 1] - M["cp"][c0]
    lo, hi = M["cp"][c0], M["cp"][c1]
    return {"vt": M["vt"], "nrow": M["nrow"], "ncol": c1 - c0, "cp": cp, "ir": M["ir"][lo:hi], "val": M["val"][lo:hi]}


def csc_rows(M, r0, r1):
    keep = (M["ir"] >= r0) & (M["ir"] < r1)
    col = np.repeat(np.arange(M["ncol"]), np.diff(M["cp"]))
    cp = np.zeros(M["ncol"] + 1, np.int64)
    np.cumsum(np.bincount(col[keep], minlength=M["ncol"]), out=cp[1:])
    return {"vt": M["vt"], "nrow": r1 - r0, "ncol": M["ncol"], "cp": cp, "ir": M["ir"][keep] - r0,
            "val": M["val"][keep]}


def main():
    if not os.path.exists(PROBE):
        sys.exit("build oracle/_ref/refprobe first (make -C oracle/ref)")
    tmp = tempfile.mkdtemp(prefix="cbmerge")
    T = lambda n: os.path.join(tmp, n)  # noqa: E731
    z = np.load(os.path.join(HERE, "g500_s10.npz"))
    n = int(z["A_shape"][0])
    A = {"vt": 1, "nrow": n, "ncol": n, "cp": z["A_cp"].astype(np.int64), "ir": z["A_ir"].astype(np.int64),
         "val": z["A_ival"].astype(np.int64)}
    out = {}
    meta = {}
    # --- split products, merged in part order
    k = 4
    cuts = [n * i // k for i in range(k + 1)]
    files = []
    for l in range(k):
        fa, fb, fc = T(f"a{l}.bin"), T(f"b{l}.bin"), T(f"p{l}.bin")
        write_cbm(fa, csc_cols(A, cuts[l], cuts[l + 1]))
        write_cbm(fb, csc_rows(A, cuts[l], cuts[l + 1]))
        probe("mult", "select2nd_i64", "hash", fa, fb, fc)
        files.append(fc)
        P = read_cbm(fc)
        out[f"split_L{l}_cp"], out[f"split_L{l}_ir"], out[f"split_L{l}_val"] = P["cp"], P["ir"].astype(np.int32), P["val"]
    for sr in ("select2nd_i64", "plus_times_i64"):
        oh, og = T("heap.bin"), T("hash.bin")
        meta[f"split_{sr}"] = probe("merge", sr, str(k), *files, oh, og)
        for tag, f in (("heap", oh), ("hash", og)):
            M = read_cbm(f)
            out[f"split_{sr}_{tag}_cp"], out[f"split_{sr}_{tag}_ir"] = M["cp"], M["ir"].astype(np.int32)
            out[f"split_{sr}_{tag}_val"] = M["val"]
    # --- random overlapping lists
    rng = np.random.default_rng(5)
    m, nc, kr = 300, 200, 3
    files = []
    for l in range(kr):
        mask = rng.random((m, nc)) < 0.08
        rows, cols = np.nonzero(mask.T)   # column-major
        cp = np.zeros(nc + 1, np.int64)
        np.cumsum(np.bincount(rows, minlength=nc), out=cp[1:])
        val = (l + 1) * 1000 + rng.integers(1, 999, len(cols))
        f = T(f"r{l}.bin")
        write_cbm(f, {"vt": 1, "nrow": m, "ncol": nc, "cp": cp, "ir": cols.astype(np.int64), "val": val})
        files.append(f)
        out[f"rand_L{l}_cp"], out[f"rand_L{l}_ir"], out[f"rand_L{l}_val"] = cp, cols.astype(np.int32), val
    for sr in ("select2nd_i64", "plus_times_i64", "min_plus_i64"):
        oh, og = T("heap.bin"), T("hash.bin")
        meta[f"rand_{sr}"] = probe("merge", sr, str(kr), *files, oh, og)
        for tag, f in (("heap", oh), ("hash", og)):
            M = read_cbm(f)
            out[f"rand_{sr}_{tag}_cp"], out[f"rand_{sr}_{tag}_ir"] = M["cp"], M["ir"].astype(np.int32)
            out[f"rand_{sr}_{tag}_val"] = M["val"]
    out["split_k"] = np.array(k)
    out["rand_k"] = np.array(kr)
    out["split_shape"] = np.array([n, n])
    out["rand_shape"] = np.array([m, nc])
    np.savez_compressed(os.path.join(HERE, "merge.npz"), **out)
    print(json.dumps(meta))


if __name__ == "__main__":
    main()
