"""GPU: the device Graph500 Kronecker generator (cbg_generate_rmat / cbg_rmat_block, kron.hip) against the
reference's own generator output (refprobe `gen` hashes in golden/kron.json, make_golden_kron.py) and
against host slices of the same matrix (the per-rank blocks of SpParMat / SpParMat3D)."""
import json
import os

import numpy as np
import pytest

import combblas_amd as cb
from combblas_amd.dist import block_range, piece_range, slice_csc
from helpers import canonical_sha256

pytestmark = pytest.mark.gpu

CASES = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "kron.json")))["cases"]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"s{c['scale']}_seed{c['seed']}")
def test_gpu_generate_rmat_matches_reference(gpu_ctx, case):
    A = gpu_ctx.generate_rmat(case["scale"], case["edgefactor"], seed=case["seed"])
    cp, ir, val = A.to_host()
    A.free()
    assert len(ir) == case["nnz"] and val.sum() == case["sum_val"]
    assert canonical_sha256(cp, ir, val) == case["sha256"]


def _blocks(n):
    out = [(0, n, 0, n), (0, 0, 0, n), (3, 3, 5, 5), (17, 901, 33, 4000), (n - 1, n, 0, 1)]
    for q in (2, 3):                       # 2D SpParMat blocks (q x q)
        for i in range(q):
            for j in range(q):
                out.append(block_range(n, q, i) + block_range(n, q, j))
    for L in (2, 3):                       # SpParMat3D pieces: colsplit and rowsplit at q = 2
        for i in range(2):
            for j in range(2):
                for l in range(L):
                    out.append(block_range(n, 2, i) + piece_range(n, 2, L, j, l))
                    out.append(piece_range(n, 2, L, i, l) + block_range(n, 2, j))
    return out


@pytest.mark.parametrize("scale,seed", [(12, cb.G500_SEED), (14, 7), (16, cb.G500_SEED)])
def test_gpu_rmat_block_matches_host_slice(gpu_ctx, scale, seed):
    n, cp, ir, val = cb.generate_rmat_host(scale, 16, seed=seed)
    for r0, r1, c0, c1 in _blocks(n):
        B = gpu_ctx.rmat_block(scale, r0, r1, c0, c1, 16, seed=seed)
        bcp, bir, bval = B.to_host()
        assert (B.getnrow(), B.getncol()) == (r1 - r0, c1 - c0)
        bval = np.zeros(0) if bval is None else bval
        B.free()
        scp, sir, sval = slice_csc(cp, ir, val, r0, r1, c0, c1)
        assert np.array_equal(bcp, scp) and np.array_equal(bir, sir) and np.array_equal(bval, sval), (r0, r1, c0, c1)


def test_gpu_rmat_block_bad_range(gpu_ctx):
    with pytest.raises(cb.CbgError) as ei:
        gpu_ctx.rmat_block(10, 0, 2000, 0, 10)
    assert ei.value.status == 3002
    with pytest.raises(cb.CbgError):
        gpu_ctx.rmat_block(10, 5, 4, 0, 10)
