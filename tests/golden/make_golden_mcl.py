#!/usr/bin/env python3
"""Generate tests/golden/mcl.npz and galerkin.npz from the REFERENCE (run in the build container).

HipMCL expansion (BASELINE config 4): a small protein-similarity-like graph
(combblas_amd.inputs.protein_like_graph, seeded) is squared by the reference's LocalSpGEMMHash and
pruned by the reference's MCLPruneRecoverySelect (ParFriends.h:185-353) under three parameter sets
that exercise the prune-only, selection and recovery branches; MemEfficientSpGEMM
(ParFriends.h:449-730) is run at 1 and 3 phases.  All through oracle/_ref/refprobe (1 MPI rank).

Galerkin triple product (BASELINE config 5): A = 3D Poisson 7-point on a 6^3 grid, R = MIS-2
aggregation (combblas_amd.inputs.aggregation_restriction); the reference's LocalSpGEMMHash computes
R^T A and then (R^T A) R (the order of RestrictionOp.cpp:188-196).

Fixture arrays: A_*, C2 (= A*A) sha/nnz, P<i>_cp/_ir/_val (pruned), P<i>_params, M<ph>_* (memeff).
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
sys.path.insert(0, REPO)
from cbm import read_cbm, write_cbm, canonical_sha256  # noqa: E402
from combblas_amd.inputs import protein_like_graph, poisson3d, aggregation_restriction  # noqa: E402

PARAMS = [(1e-4, 1100, 1400, 0.9),   # MCL defaults (Applications/MCL.cpp:147-151): prune only here
          (1e-3, 40, 60, 0.9),       # selection, recovery after selection
          (0.02, 30, 50, 0.95)]      # recovery


def probe(*args):
    out = subprocess.run([PROBE, *map(str, args)], check=True, capture_output=True, text=True).stdout
    lines = [l for l in out.splitlines() if l.startswith("{")]
    return json.loads(lines[-1]) if lines else {}


def cbm(path, nrow, ncol, cp, ir, val):
    write_cbm(path, {"vt": 0, "nrow": nrow, "ncol": ncol, "cp": cp, "ir": ir, "val": val})


def main():
    tmp = tempfile.mkdtemp(prefix="cbmcl")
    T = lambda n: os.path.join(tmp, n)  # noqa: E731
    man = {}
    # ---------------------------------------------------------------- HipMCL expansion
    n, cp, ir, val = protein_like_graph(1200, seed=7, cmin=20, cmax=150, density=0.2, noise=2e-4)
    fa = T("a.bin")
    cbm(fa, n, n, cp, ir, val)
    fc = T("c2.bin")
    info = probe("mult", "plus_times_f64", "hash", fa, fa, fc)
    C2 = read_cbm(fc)
    d = {"A_cp": cp, "A_ir": ir, "A_val": val, "A_shape": np.array([n, n], np.int64),
         "C2_nnz": np.array(len(C2["ir"]), np.int64), "C2_flops": np.array(info["flops"], np.int64),
         "C2_sha256": np.array(canonical_sha256(C2["cp"], C2["ir"], C2["val"]))}
    for i, (thr, sel, rec, pct) in enumerate(PARAMS):
        fo = T(f"p{i}.bin")
        probe("mcl", fc, repr(thr), sel, rec, repr(pct), fo)
        P = read_cbm(fo)
        d[f"P{i}_cp"], d[f"P{i}_ir"], d[f"P{i}_val"] = P["cp"], P["ir"].astype(np.int32), P["val"]
        d[f"P{i}_params"] = np.array([thr, sel, rec, pct], np.float64)
        man[f"P{i}"] = {"params": [thr, sel, rec, pct], "nnz": int(len(P["ir"]))}
    thr, sel, rec, pct = PARAMS[1]
    for ph in (1, 3):
        fo = T(f"m{ph}.bin")
        probe("memeff", fa, ph, repr(thr), sel, rec, repr(pct), fo)
        M = read_cbm(fo)
        d[f"M{ph}_cp"], d[f"M{ph}_ir"], d[f"M{ph}_val"] = M["cp"], M["ir"].astype(np.int32), M["val"]
        man[f"M{ph}"] = {"phases": ph, "params": [thr, sel, rec, pct], "nnz": int(len(M["ir"]))}
    np.savez_compressed(os.path.join(HERE, "mcl.npz"), **d)
    man["C2"] = {"nnz": int(len(C2["ir"])), "flops": info["flops"]}
    # ---------------------------------------------------------------- Galerkin R^T A R
    n, acp, air, aval = poisson3d(6)
    nagg, rcp, rir, rval = aggregation_restriction(n, acp, air, seed=3)
    import scipy.sparse as sp
    Rt = sp.csc_matrix((rval, rir, rcp), shape=(n, nagg)).T.tocsc()
    Rt.sort_indices()
    fA, fR, fRt = T("ga.bin"), T("gr.bin"), T("grt.bin")
    cbm(fA, n, n, acp, air, aval)
    cbm(fR, n, nagg, rcp, rir, rval)
    cbm(fRt, nagg, n, Rt.indptr.astype(np.int64), Rt.indices.astype(np.int64), Rt.data)
    fRA, fC = T("gra.bin"), T("gc.bin")
    i1 = probe("mult", "plus_times_f64", "hash", fRt, fA, fRA)
    i2 = probe("mult", "plus_times_f64", "hash", fRA, fR, fC)
    RA, Cg = read_cbm(fRA), read_cbm(fC)
    np.savez_compressed(os.path.join(HERE, "galerkin.npz"),
                        A_cp=acp, A_ir=air, A_val=aval, A_shape=np.array([n, n], np.int64),
                        R_cp=rcp, R_ir=rir, R_val=rval, R_shape=np.array([n, nagg], np.int64),
                        RA_cp=RA["cp"], RA_ir=RA["ir"].astype(np.int32), RA_val=RA["val"],
                        C_cp=Cg["cp"], C_ir=Cg["ir"].astype(np.int32), C_val=Cg["val"],
                        RA_flops=np.array(i1["flops"], np.int64), C_flops=np.array(i2["flops"], np.int64))
    man["galerkin"] = {"n": n, "nagg": nagg, "RA_nnz": int(len(RA["ir"])), "C_nnz": int(len(Cg["ir"]))}
    mp = os.path.join(HERE, "MANIFEST.json")
    M = json.load(open(mp))
    M["mcl_galerkin"] = {"generator": "tests/golden/make_golden_mcl.py via oracle/_ref/refprobe", **man}
    json.dump(M, open(mp, "w"), indent=1)
    print(json.dumps(man))


if __name__ == "__main__":
    main()
