#!/usr/bin/env python3
"""Diagnose a sampled-column mismatch of the R-MAT product against the oracle (GPU box).

    python tools/diag_s20.py [scale] [stride] [out.json]

Computes A*A on the device (whatever libcbgpu CBG_LIB_PATH names), the oracle product of every
stride-th column, and reports the differing columns with their statistics (flops, B nnz, span,
heavy or not, how the rows differ).  Test infrastructure only.
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests"))

import combblas_amd as cb  # noqa: E402
from helpers import Csc, oracle_spgemm  # noqa: E402


def main():
    scale = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    stride = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    out = sys.argv[3] if len(sys.argv) > 3 else None
    n, cp, ir, val = cb.generate_rmat_host(scale, 16, seed=1)
    ctx = cb.Context(0)
    dA = cb.SpDCCols.from_csc(ctx, n, n, cp, ir, val)
    t = time.time()
    C = cb.LocalSpGEMMHash(cb.PlusTimesSRing("f64"), dA, dA)
    prof = ctx.last_profile()
    print(f"product nnz {C.getnnz()} in {time.time() - t:.2f}s bins {prof['bins']}", flush=True)
    cols = np.arange(0, n, stride)
    alen = np.diff(cp)
    sel = np.concatenate([np.arange(cp[c], cp[c + 1]) for c in cols])
    B = Csc(n, len(cols), np.r_[0, np.cumsum(alen[cols])], ir[sel], val[sel])
    R, rm, rc = oracle_spgemm(Csc(n, n, cp, ir, val), B, "plus_times", "f64")
    try:
        S = C.select_columns(cols)
        scp, sir, sval = S.to_host()
    except AttributeError:   # a variant library without cbg_col_select: select on the host
        fcp, fir, fval = C.to_host()
        idx = np.concatenate([np.arange(fcp[c], fcp[c + 1]) for c in cols])
        scp = np.r_[0, np.cumsum(np.diff(fcp)[cols])]
        sir, sval = fir[idx], fval[idx]
        del fir, fval
    gn, rn = np.diff(scp), np.diff(R.cp)
    bad_cnt = np.flatnonzero(gn != rn)
    bad_rows, bad_vals = [], []
    for t_, j in enumerate(cols):
        if gn[t_] != rn[t_]:
            continue
        a, b = scp[t_], R.cp[t_]
        g, r = sir[a:a + gn[t_]], R.ir[b:b + rn[t_]]
        if not np.array_equal(g, r):
            bad_rows.append(t_)
        elif not np.array_equal(sval[a:a + gn[t_]], R.val[b:b + rn[t_]]):
            bad_vals.append(t_)
    flop = np.bincount(np.repeat(np.arange(n), alen), weights=alen[ir], minlength=n).astype(np.int64)
    rep = {"scale": scale, "stride": stride, "columns": int(len(cols)), "nnz_gpu": int(scp[-1]), "nnz_orc": int(R.cp[-1]),
           "bad_count_cols": int(len(bad_cnt)), "bad_row_cols": len(bad_rows), "bad_val_cols": len(bad_vals),
           "lib": os.environ.get("CBG_LIB_PATH", "in-tree"), "examples": []}
    for t_ in list(bad_cnt[:12]) + bad_rows[:6] + bad_vals[:6]:
        j = int(cols[t_])
        a, b = scp[t_], R.cp[t_]
        g, r = sir[a:a + gn[t_]], R.ir[b:b + rn[t_]]
        ks = ir[cp[j]:cp[j + 1]]
        lo = min((ir[cp[k]] for k in ks if alen[k]), default=-1)
        hi = max((ir[cp[k + 1] - 1] for k in ks if alen[k]), default=-1)
        ex = {"col": j, "nnz_gpu": int(gn[t_]), "nnz_orc": int(rn[t_]), "flop": int(flop[j]), "nb": int(len(ks)),
              "span": [int(lo), int(hi)], "heavy": bool(rn[t_] > 4096)}
        if gn[t_] == rn[t_] and not np.array_equal(g, r):
            d = np.flatnonzero(g != r)
            ex["first_row_diff"] = [int(d[0]), int(g[d[0]]), int(r[d[0]])]
        elif gn[t_] != rn[t_]:
            sg, sr_ = set(g.tolist()), set(r.tolist())
            miss, extra = sorted(sr_ - sg), sorted(sg - sr_)
            ex["missing"] = [int(x) for x in miss[:10]] + ([len(miss)] if len(miss) > 10 else [])
            ex["extra"] = [int(x) for x in extra[:10]] + ([len(extra)] if len(extra) > 10 else [])
            ex["gpu_sorted"] = bool(np.all(np.diff(g) > 0))
            ex["gpu_dups"] = int(len(g) - len(np.unique(g)))
        else:
            d = np.flatnonzero(sval[a:a + gn[t_]] != R.val[b:b + rn[t_]])
            ex["val_diffs"] = int(len(d))
            ex["first_val_diff"] = [int(g[d[0]]), float(sval[a + d[0]]), float(R.val[b + d[0]])]
        rep["examples"].append(ex)
    print(json.dumps(rep, indent=1))
    if out:
        json.dump(rep, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
