"""CPU: the oracle's MCLPruneRecoverySelect restatement reproduces the reference's own outputs
(tests/golden/mcl.npz, made by oracle/_ref/refprobe from ParFriends.h:185-353 and :449-730), and the
config-4/5 input generators behave.  Galerkin fixtures: the oracle SpGEMM reproduces R^T A and
(R^T A) R (RestrictionOp.cpp:188-196 order) computed by the reference's LocalSpGEMMHash."""
import numpy as np
import pytest

from helpers import Csc, load_fixture, oracle_mcl_prune, oracle_spgemm, assert_same_product, canonical_sha256


def _mcl_inputs():
    z = load_fixture("mcl")
    n = int(z["A_shape"][0])
    A = Csc(n, n, z["A_cp"], z["A_ir"], z["A_val"])
    C2, mults, rc = oracle_spgemm(A, A, "plus_times", "f64")
    assert rc == 0
    return z, A, C2, mults


def test_oracle_square_matches_reference():
    z, A, C2, mults = _mcl_inputs()
    assert mults == int(z["C2_flops"])
    assert C2.nnz == int(z["C2_nnz"])
    assert canonical_sha256(C2.cp, C2.ir, C2.val) == str(z["C2_sha256"])


@pytest.mark.parametrize("i", [0, 1, 2])
def test_oracle_prune_matches_reference(i):
    z, A, C2, _ = _mcl_inputs()
    thr, sel, rec, pct = z[f"P{i}_params"]
    P, st = oracle_mcl_prune(C2, float(thr), int(sel), int(rec), float(pct))
    R = Csc(C2.nrow, C2.ncol, z[f"P{i}_cp"], z[f"P{i}_ir"], z[f"P{i}_val"])
    assert_same_product(P, R, "f64", rtol=0.0, what=f"P{i}")
    if i == 1:
        assert st[1] > 0 and st[2] > 0, st   # selection and recovery-after-selection exercised
    if i == 2:
        assert st[0] > 0, st                 # recovery exercised


@pytest.mark.parametrize("ph", [1, 3])
def test_memeff_phases_equal_prune_of_product(ph):
    """MemEfficientSpGEMM output is phase-count independent: prune(A*A) column by column."""
    z, A, C2, _ = _mcl_inputs()
    thr, sel, rec, pct = z["P1_params"]
    R = Csc(C2.nrow, C2.ncol, z[f"M{ph}_cp"], z[f"M{ph}_ir"], z[f"M{ph}_val"])
    P, _ = oracle_mcl_prune(C2, float(thr), int(sel), int(rec), float(pct))
    assert_same_product(P, R, "f64", rtol=0.0, what=f"memeff phases={ph}")


def test_oracle_galerkin_matches_reference():
    z = load_fixture("galerkin")
    n, nagg = (int(x) for x in z["R_shape"])
    A = Csc(n, n, z["A_cp"], z["A_ir"], z["A_val"])
    R = Csc(n, nagg, z["R_cp"], z["R_ir"], z["R_val"])
    Rt = Csc(nagg, n, *_transpose(R))
    RA, m1, _ = oracle_spgemm(Rt, A, "plus_times", "f64")
    C, m2, _ = oracle_spgemm(RA, R, "plus_times", "f64")
    assert (m1, m2) == (int(z["RA_flops"]), int(z["C_flops"]))
    assert_same_product(RA, Csc(nagg, n, z["RA_cp"], z["RA_ir"], z["RA_val"]), "f64", what="R^T A")
    assert_same_product(C, Csc(nagg, nagg, z["C_cp"], z["C_ir"], z["C_val"]), "f64", what="R^T A R")


def _transpose(M):
    import scipy.sparse as sp
    T = sp.csc_matrix((M.val, M.ir, M.cp), shape=(M.nrow, M.ncol)).T.tocsc()
    T.sort_indices()
    return T.indptr.astype(np.int64), T.indices.astype(np.int32), T.data


def test_generators():
    from combblas_amd.inputs import protein_like_graph, poisson3d, aggregation_restriction
    n, cp, ir, val = protein_like_graph(500, seed=3, cmax=100)
    sums = np.add.reduceat(val, cp[:-1])
    assert np.allclose(sums, 1.0) and np.all(val > 0)
    n2, cp2, ir2, val2 = protein_like_graph(500, seed=3, cmax=100)
    assert np.array_equal(ir, ir2) and np.array_equal(val, val2)
    n, acp, air, aval = poisson3d(4)
    rs = np.add.reduceat(aval, acp[:-1])
    assert n == 64 and acp[-1] == 64 + 2 * 3 * (3 * 4 * 4) and rs.min() == 0.0 and rs.max() == 3.0
    nagg, rcp, rir, rval = aggregation_restriction(n, acp, air, seed=1)
    assert rcp[-1] == n and 1 < nagg < n
    rows = np.sort(rir)
    assert np.array_equal(rows, np.arange(n))   # every vertex in exactly one aggregate
