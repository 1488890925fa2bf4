#!/usr/bin/env python3
"""cbg_merge (MultiwayMergeHash, MultiwayMerge.h:536-684) at the 1x1x2 layout's sizes on one GPU.

The two partials are the layer products of the 1x1x2 grid: P_l = A[:, K_l] * B[K_l, :] with the inner
dimension cut in half, every operand piece built on the device (cbg_rmat_block); the merge of P_0 and
P_1 is timed (HIP-synchronised wall clock per call) and reported with SURVEY §8(d)'s merge bytes
sum nnz(partials) * (s_i + s_v) * 2 + nnz(C) * (s_i + s_v).
usage: python tools/bench_merge.py [--scale S] [--reps R]
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=19)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--lib", default=None, help="another libcbgpu.so (a tools/var build)")
    a = ap.parse_args()
    from combblas_amd import _abi
    if a.lib:
        _abi.LIB_PATH = os.path.abspath(a.lib)
    import combblas_amd as cb
    ctx = cb.Context(0)
    PT = cb.PlusTimesSRing("f64")
    n = 1 << a.scale
    h = n // 2
    parts = []
    for (k0, k1) in ((0, h), (h, n)):
        Ak = ctx.rmat_block(a.scale, 0, n, k0, k1)
        Bk = ctx.rmat_block(a.scale, k0, k1, 0, n)
        parts.append(cb.LocalSpGEMMHash(PT, Ak, Bk))
        Ak.free()
        Bk.free()
    ts = []
    for _ in range(a.reps + 1):
        ctx.synchronize()
        t0 = time.perf_counter()
        C = ctx.merge(parts, PT)
        ctx.synchronize()
        ts.append(time.perf_counter() - t0)
        nnzc = C.getnnz()
        C.free()
    t = min(ts[1:])
    nparts = [p.getnnz() for p in parts]
    # merged positions per column (the two-way merge walks one column per wave): how skewed is the work?
    import numpy as np
    import ctypes

    def colptr(p):   # the colptr alone (rows and values stay on the device)
        cp = np.empty(p.getncol() + 1, np.int64)
        _abi.check(ctx._lib.cbg_result_to_host(ctx._ptr, ctypes.byref(p._res), cp.ctypes.data, None, None), "colptr")
        return cp
    lens = sum(np.diff(colptr(p)) for p in parts)
    tail = {"max_column_positions": int(lens.max()), "columns_over_16k": int((lens > 16384).sum()),
            "positions_in_columns_over_16k": int(lens[lens > 16384].sum()), "positions": int(lens.sum())}
    byts = sum(nparts) * 12 * 2 + nnzc * 12
    print(json.dumps({"what": "cbg_merge of the two 1x1x2 layer partials", "scale": a.scale, "lib": a.lib,
                      "nnz_partials": nparts, "nnz_C": nnzc, "merge_ms": t * 1e3,
                      "merge_bytes": byts, "merge_GBps": byts / t / 1e9, "reps_ms": [x * 1e3 for x in ts],
                      "column_skew": tail}),
          flush=True)


if __name__ == "__main__":
    main()
