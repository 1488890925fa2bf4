#!/usr/bin/env python3
"""Reference-generated Graph500 Kronecker matrices pinned by hash -> tests/golden/kron.json.

Runs oracle/_ref/refprobe `gen` (DistEdgeList::GenGraph500Data(packed=true) + SpParMat(DEL, false),
oracle/ref/refprobe.cpp run_gen; the reference's own SEED default 0xDECAFBAD, or SEED=<s> in the
environment as RefGen21::init_random reads it) at scales 10-18 and records, per (scale, seed), nnz and
the canonical SHA-256 of the column-sorted CSC (cbm.canonical_sha256).  The s10 / s12 matrices are
also stored whole in g500_s10.npz / g500_s12.npz (make_golden.py).

    python tests/golden/make_golden_kron.py     # in the build container (needs /root/reference)
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
from cbm import canonical_sha256, read_cbm  # noqa: E402

PROBE = os.path.join(REPO, "oracle", "_ref", "refprobe")
CASES = [(s, None) for s in (10, 12, 14, 16, 18, 20)] + [(12, 1), (14, 7)]


def main():
    if not os.path.exists(PROBE):
        sys.exit("build oracle/_ref/refprobe first (make -C oracle/ref)")
    out = []
    with tempfile.TemporaryDirectory() as td:
        for scale, seed in CASES:
            env = dict(os.environ)
            env.pop("SEED", None)
            if seed is not None:
                env["SEED"] = str(seed)
            path = os.path.join(td, f"g{scale}.cbm")
            subprocess.run([PROBE, "gen", str(scale), "16", path], check=True, env=env, stdout=subprocess.DEVNULL)
            M = read_cbm(path)
            out.append({"scale": scale, "edgefactor": 16, "seed": 0xDECAFBAD if seed is None else seed,
                        "nnz": int(len(M["ir"])), "sum_val": float(np.sum(M["val"])),
                        "sha256": canonical_sha256(M["cp"], M["ir"].astype(np.int32), M["val"])})
            print(out[-1], flush=True)
    json.dump({"generator": "tests/golden/make_golden_kron.py via oracle/_ref/refprobe gen",
               "reference": "DistEdgeList.cpp:223-280 (packed), RefGen21.h:102-318, SpParMat.cpp:3082-3196",
               "cases": out}, open(os.path.join(HERE, "kron.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
