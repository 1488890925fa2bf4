#!/usr/bin/env python3
"""One-GPU measurements of BASELINE configs 4 and 5 (the bench line is config 2, bench.py).

  config 4  HipMCL expansion: A*A of a protein-similarity-like graph (combblas_amd.inputs), then
            MCLPruneRecoverySelect with MCL's defaults -- MemEfficientSpGEMM (ParFriends.h:449-730).
  config 5  Galerkin triple product R^T A R: A = 3D Poisson 7-point on k^3, R = MIS-2 aggregation,
            computed as (R^T A) R (RestrictionOp.cpp:188-196 order).
Inputs are generated on the host and uploaded before timing; each timed region is whole library
calls (device work + the host syncs they contain).  Prints one JSON object per config.
usage: python tools/bench_configs.py [--mcl-n N] [--poisson-k K] [--reps R]
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402

import combblas_amd as cb  # noqa: E402
from combblas_amd.inputs import poisson3d, protein_like_graph  # noqa: E402


def timed(ctx, fn, reps):
    fn()                       # warm-up (pool, code objects)
    ctx.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        ctx.synchronize()
        ts.append(time.perf_counter() - t0)
        if out is not None and hasattr(out, "free"):
            out.free()
    return float(np.median(ts))


def transpose_csc(nrow, ncol, cp, ir, val):
    import scipy.sparse as sp
    T = sp.csc_matrix((val, ir, cp), shape=(nrow, ncol)).T.tocsc()
    T.sort_indices()
    return T.indptr.astype(np.int64), T.indices.astype(np.int32), T.data


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mcl-n", type=int, default=1 << 18)
    ap.add_argument("--poisson-k", type=int, default=128)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--only", type=int, default=0, help="run only config 4 or 5")
    args = ap.parse_args()
    ctx = cb.Context(0)
    PT = cb.PlusTimesSRing("f64")

    # ---------------------------------------------------------------- config 4
    if args.only in (0, 4):
        config4(ctx, PT, args)
    if args.only in (0, 5):
        config5(ctx, PT, args)


def config4(ctx, PT, args):
    t0 = time.perf_counter()
    n, cp, ir, val = protein_like_graph(args.mcl_n, seed=1)
    gen_s = time.perf_counter() - t0
    A = cb.SpDCCols.from_csc(ctx, n, n, cp, ir, val)
    d = cb.MCL_DEFAULTS
    stats = {}
    C = cb.MemEfficientSpGEMM(PT, A, A, 1, d["hardThreshold"], d["selectNum"], d["recoverNum"], d["recoverPct"],
                              stats=stats)
    nnz_pruned = C.getnnz()
    C.free()
    t_exp = timed(ctx, lambda: cb.MemEfficientSpGEMM(PT, A, A, 1, d["hardThreshold"], d["selectNum"],
                                                     d["recoverNum"], d["recoverPct"]), args.reps)
    t_mul = timed(ctx, lambda: cb.LocalSpGEMMHash(PT, A, A), args.reps)
    mults = stats["multiplies"]
    print(json.dumps({"config": "4: HipMCL expansion A*A + MCLPruneRecoverySelect (MCL defaults), 1 GPU",
                      "graph": {"n": n, "nnz": int(cp[-1]), "clusters": "log-uniform [20, 2000]", "density": 0.2,
                                "noise": 1e-5, "gen_s": round(gen_s, 2)},
                      "multiplies": mults, "nnz_product": stats["nnz_unpruned"], "nnz_pruned": nnz_pruned,
                      "branches": {k: stats[k] for k in ("recovered", "selected", "recovered_after_select")},
                      "expansion_ms": t_exp * 1e3, "product_ms": t_mul * 1e3, "prune_ms": (t_exp - t_mul) * 1e3,
                      "multiplies_per_s": mults / t_exp, "unit": "multiplies/s"}), flush=True)
    A.free()


def config5(ctx, PT, args):
    t0 = time.perf_counter()
    n, acp, air, aval = poisson3d(args.poisson_k)
    gen_s = time.perf_counter() - t0
    dA = cb.SpDCCols.from_csc(ctx, n, n, acp, air, aval)
    ctx.synchronize()
    t0 = time.perf_counter()
    dR, dRt = cb.RestrictionOp(dA)          # the reference's RestrictionOp on the device (galerkin.hip)
    ctx.synchronize()
    r_s = time.perf_counter() - t0
    nagg = dR.getncol()

    class _Pair:   # both restriction outputs, freed together by timed()
        def __init__(self, rr):
            self.rr = rr

        def free(self):
            for m in self.rr:
                m.free()

    t_restrict = timed(ctx, lambda: _Pair(cb.RestrictionOp(dA)), args.reps)
    t_fast = timed(ctx, lambda: _Pair(cb.MIS2Restriction(dA, seed=1)), args.reps)
    RA = cb.LocalSpGEMMHash(PT, dRt, dA)
    C = cb.LocalSpGEMMHash(PT, RA, dR)
    m1, m2, nnz_ra, nnz_c = RA.multiplies, C.multiplies, RA.getnnz(), C.getnnz()
    RA.free()
    C.free()

    def triple():
        ra = cb.LocalSpGEMMHash(PT, dRt, dA)
        c = cb.LocalSpGEMMHash(PT, ra, dR)
        ra.free()
        return c

    def fused():
        return cb.GalerkinRAP(dA, dR)

    t_gal = timed(ctx, triple, args.reps)
    t_fused = timed(ctx, fused, args.reps)
    print(json.dumps({"config": "5: Galerkin R^T A R, 3D Poisson 7-point, the reference's RestrictionOp R (device), 1 GPU",
                      "A": {"k": args.poisson_k, "n": n, "nnz": int(acp[-1])}, "R": {"nagg": nagg},
                      "gen_s": round(gen_s, 2), "restriction_device_ms": round(t_restrict * 1e3, 3),
                      "restriction_first_call_ms": round(r_s * 1e3, 3),
                      "restriction_note": "RestrictionOp = the reference's R (MTRand MIS2, Select2ndRandSR, RandPerm); "
                                          "MIS2Restriction = hash-priority Luby MIS-2 (not the reference's R)",
                      "mis2_fast_ms": round(t_fast * 1e3, 3),
                      "multiplies": m1 + m2, "nnz_RtA": nnz_ra, "nnz_C": nnz_c,
                      "triple_ms": t_gal * 1e3, "multiplies_per_s": (m1 + m2) / t_gal, "unit": "multiplies/s",
                      "fused_rap_ms": t_fused * 1e3,
                      "fused_note": "cbg_galerkin_rap: per-aggregate LDS sort-and-sum over nnz(A) (one pass) + compaction; "
                                    "multiplies_per_s above counts the two-product work at the two-product time"}),
          flush=True)


if __name__ == "__main__":
    main()
