"""GPU parity of the HipMCL expansion (BASELINE config 4) and the Galerkin triple product (config 5).

cbg_mcl_prune / MemEfficientSpGEMM / cbg_col_range / cbg_col_concat through the C ABI against
  * the reference's own outputs (tests/golden/mcl.npz, galerkin.npz; oracle/_ref/refprobe), and
  * the oracle's MCLPruneRecoverySelect restatement on larger seeded graphs.
Bars: structure exact; pruned values are the product's values (PlusTimes<double>: <= 1e-12 rel).
The prune itself is checked bit-exact by feeding the oracle the GPU's own product.
"""
import numpy as np
import pytest

import combblas_amd as cb
from combblas_amd import mcl as cmcl
from combblas_amd.inputs import aggregation_restriction, poisson3d, protein_like_graph
from helpers import Csc, assert_same_product, load_fixture, oracle_mcl_prune, oracle_spgemm

pytestmark = pytest.mark.gpu
PT = cb.PlusTimesSRing("f64")


def up(ctx, M, dtype=None):
    return cb.SpDCCols.from_csc(ctx, M.nrow, M.ncol, M.cp, M.ir, M.val, dtype=dtype)


def host(M, nrow):
    cp, ir, val = M.to_host()
    return Csc(nrow, len(cp) - 1, cp, ir, val)


def mcl_fixture():
    z = load_fixture("mcl")
    n = int(z["A_shape"][0])
    return z, Csc(n, n, z["A_cp"], z["A_ir"], z["A_val"])


@pytest.mark.parametrize("i", [0, 1, 2])
def test_prune_matches_reference(gpu_ctx, i):
    z, A = mcl_fixture()
    thr, sel, rec, pct = (float(x) for x in z[f"P{i}_params"])
    dA = up(gpu_ctx, A)
    C = cb.LocalSpGEMMHash(PT, dA, dA)
    Ch = host(C, A.nrow)
    st = cb.MCLPruneRecoverySelect(C, thr, int(sel), int(rec), pct)
    P = host(C, A.nrow)
    R = Csc(A.nrow, A.ncol, z[f"P{i}_cp"], z[f"P{i}_ir"], z[f"P{i}_val"])
    assert_same_product(P, R, "f64", what=f"P{i} vs reference")
    O, ost = oracle_mcl_prune(Ch, thr, int(sel), int(rec), pct)
    assert_same_product(P, O, "f64", rtol=0.0, what=f"P{i} vs oracle")
    assert (st["recovered"], st["selected"], st["recovered_after_select"]) == ost


@pytest.mark.parametrize("ph", [1, 3])
def test_memeff_matches_reference(gpu_ctx, ph):
    z, A = mcl_fixture()
    thr, sel, rec, pct = (float(x) for x in z["P1_params"])
    dA = up(gpu_ctx, A)
    stats = {}
    C = cb.MemEfficientSpGEMM(PT, dA, dA, ph, thr, int(sel), int(rec), pct, stats=stats)
    assert stats["phases"] == ph and stats["multiplies"] == int(z["C2_flops"])
    R = Csc(A.nrow, A.ncol, z[f"M{ph}_cp"], z[f"M{ph}_ir"], z[f"M{ph}_val"])
    assert_same_product(host(C, A.nrow), R, "f64", what=f"memeff phases={ph}")


@pytest.mark.parametrize("n,seed,params", [
    (20000, 11, (1e-4, 1100, 1400, 0.9)),     # MCL defaults
    (20000, 12, (1e-3, 50, 80, 0.9)),         # selection-heavy
    (8000, 13, (0.05, 20, 40, 0.99)),         # recovery-heavy
])
def test_prune_matches_oracle_large(gpu_ctx, n, seed, params):
    thr, sel, rec, pct = params
    n, cp, ir, val = protein_like_graph(n, seed=seed, cmin=20, cmax=600, density=0.2, noise=1e-5)
    A = Csc(n, n, cp, ir, val)
    dA = up(gpu_ctx, A)
    C = cb.LocalSpGEMMHash(PT, dA, dA)
    Ch = host(C, n)
    st = cb.MCLPruneRecoverySelect(C, thr, sel, rec, pct)
    O, ost = oracle_mcl_prune(Ch, thr, sel, rec, pct)
    assert_same_product(host(C, n), O, "f64", rtol=0.0, what="prune vs oracle")
    assert (st["recovered"], st["selected"], st["recovered_after_select"]) == ost


def test_memeff_phases_large(gpu_ctx):
    n, cp, ir, val = protein_like_graph(30000, seed=5, cmin=20, cmax=800)
    A = Csc(n, n, cp, ir, val)
    dA = up(gpu_ctx, A)
    outs = []
    for ph in (1, 4, 7):
        C = cb.MemEfficientSpGEMM(PT, dA, dA, ph, 1e-3, 60, 90, 0.9)
        outs.append(host(C, n))
    for o in outs[1:]:   # pruning is per column, so the phase count cannot change the result
        assert np.array_equal(o.cp, outs[0].cp) and np.array_equal(o.ir, outs[0].ir)
        # LDS atomic accumulation makes f64 sums order-dependent: values agree to the 1e-12 bar
        assert np.allclose(o.val, outs[0].val, rtol=1e-12, atol=0)


def test_prune_edge_cases(gpu_ctx):
    # columns: empty; all <= thr (recovery -> keep all); fewer than select; ties at the k-th value;
    # negative values; an entry exactly equal to thr (kept by the final PruneColumn, v < thr drops)
    cols = [[], [0.001, 0.002], [0.5, 0.4], [0.3, 0.3, 0.3, 0.3, 0.1], [-1.0, 2.0, 0.5, 0.25], [0.01, 0.5, 0.49]]
    cp = np.cumsum([0] + [len(c) for c in cols]).astype(np.int64)
    ir = np.concatenate([np.arange(len(c)) for c in cols]).astype(np.int32)
    val = np.concatenate([np.array(c, np.float64) for c in cols])
    M = Csc(8, len(cols), cp, ir, val)
    for params in [(0.01, 2, 3, 0.9), (0.01, 0, 0, 0.9), (0.3, 1, 0, 0.5), (1e-4, 3, 5, 0.99)]:
        D = up(gpu_ctx, M)
        st = cb.MCLPruneRecoverySelect(D, *params)
        O, ost = oracle_mcl_prune(M, *params)
        assert_same_product(host(D, 8), O, "f64", rtol=0.0, what=f"edge {params}")
        assert (st["recovered"], st["selected"], st["recovered_after_select"]) == ost


def test_prune_selection_adversarial(gpu_ctx):
    """Columns that stress k_mcl_fused's one-histogram selection (block_kth2): one repeated value (empty key
    range), a few values with thousands of ties (gathered bucket lists overflow -> radix fallback), a column
    longer than the LDS stage (values read from HBM), values a few ulps apart (every bucket exact), mixed
    signs, and a tie block straddling the k-th position."""
    rng = np.random.default_rng(7)
    cols = [np.full(3000, 0.25),
            rng.choice([0.1, 0.2, 0.3, 0.4, 0.5], 3000),
            rng.lognormal(-6, 2, 5000),
            0.5 + np.arange(2000) * np.spacing(0.5),
            rng.normal(0, 1, 2500),
            np.concatenate([np.full(1200, 0.3), rng.uniform(0, 0.29, 300)]),
            rng.lognormal(-4, 1, 1300)]
    cols = [rng.permutation(c) for c in cols]
    cp = np.cumsum([0] + [len(c) for c in cols]).astype(np.int64)
    ir = np.concatenate([np.sort(rng.choice(6000, len(c), replace=False)) for c in cols]).astype(np.int32)
    val = np.concatenate(cols).astype(np.float64)
    M = Csc(6000, len(cols), cp, ir, val)
    for params in [(1e-4, 1100, 1400, 0.9), (1e-4, 1000, 0, 0.9), (0.6, 100, 2600, 0.99), (1e-9, 1250, 1250, 1.0),
                   (1e-9, 100, 2600, 1e6), (1e-9, 100, 1200, 1e6)]:
        D = up(gpu_ctx, M)
        st = cb.MCLPruneRecoverySelect(D, *params)
        O, ost = oracle_mcl_prune(M, *params)
        assert_same_product(host(D, 6000), O, "f64", rtol=0.0, what=f"adversarial {params}")
        assert (st["recovered"], st["selected"], st["recovered_after_select"]) == ost


def test_prune_f32_and_empty(gpu_ctx):
    n, cp, ir, val = protein_like_graph(3000, seed=2, cmax=200)
    A32 = Csc(n, n, cp, ir, val.astype(np.float32))
    D = up(gpu_ctx, A32)
    C = cb.LocalSpGEMMHash(cb.PlusTimesSRing("f32"), D, D)
    cp2, ir2, v2 = C.to_host()
    W = Csc(n, n, cp2, ir2, v2.astype(np.float64))   # f32 values widened exactly
    # rules that involve no float sums (pure threshold; selection without recovery) are exact in f32
    for (thr, sel, rec) in ((1e-3, 0, 0), (1e-3, 30, 0)):
        D2 = cb.SpDCCols._from_result(gpu_ctx, cmcl._col_range(gpu_ctx, C._res, 0, n))
        cb.MCLPruneRecoverySelect(D2, thr, sel, rec, 0.9)
        cp3, ir3, v3 = D2.to_host()
        O, _ = oracle_mcl_prune(W, float(np.float32(thr)), sel, rec, 0.9)
        assert np.array_equal(cp3, O.cp) and np.array_equal(ir3, O.ir)
        assert np.array_equal(v3.astype(np.float64), O.val)
    E = up(gpu_ctx, Csc(5, 4, np.zeros(5, np.int64), np.zeros(0, np.int32), np.zeros(0)))
    st = cb.MCLPruneRecoverySelect(E, 1e-4, 10, 20, 0.9)
    assert E.getnnz() == 0 and st["nnz_out"] == 0


def test_col_range_concat_roundtrip(gpu_ctx):
    n, cp, ir, val = protein_like_graph(2000, seed=4, cmax=100)
    D = up(gpu_ctx, Csc(n, n, cp, ir, val))
    ranges = cmcl.phase_ranges(n, 7)
    parts = [cmcl._col_range(gpu_ctx, D._res, c0, c1) for (c0, c1) in ranges]
    for (c0, c1), p in zip(ranges, parts):
        assert p.ncol == c1 - c0 and p.nnz == cp[c1] - cp[c0]
    out = cmcl._col_concat(gpu_ctx, parts)
    for p in parts:
        gpu_ctx._lib.cbg_result_free(gpu_ctx._ptr, __import__("ctypes").byref(p))
    R = cb.SpDCCols._from_result(gpu_ctx, out)
    cp2, ir2, v2 = R.to_host()
    assert np.array_equal(cp2, cp) and np.array_equal(ir2, ir) and np.array_equal(v2, val)
    with pytest.raises(cb.CbgError):
        cmcl._col_range(gpu_ctx, D._res, 5, n + 1)


def _transpose(M):
    import scipy.sparse as sp
    T = sp.csc_matrix((M.val, M.ir, M.cp), shape=(M.nrow, M.ncol)).T.tocsc()
    T.sort_indices()
    return Csc(M.ncol, M.nrow, T.indptr, T.indices, T.data)


def test_galerkin_matches_reference(gpu_ctx):
    z = load_fixture("galerkin")
    n, nagg = (int(x) for x in z["R_shape"])
    A = Csc(n, n, z["A_cp"], z["A_ir"], z["A_val"])
    R = Csc(n, nagg, z["R_cp"], z["R_ir"], z["R_val"])
    RA = cb.LocalSpGEMMHash(PT, up(gpu_ctx, _transpose(R)), up(gpu_ctx, A))
    C = cb.LocalSpGEMMHash(PT, RA, up(gpu_ctx, R))
    assert (RA.multiplies, C.multiplies) == (int(z["RA_flops"]), int(z["C_flops"]))
    assert_same_product(host(C, nagg), Csc(nagg, nagg, z["C_cp"], z["C_ir"], z["C_val"]), "f64", what="RtAR")


def test_galerkin_large_vs_oracle(gpu_ctx):
    n, acp, air, aval = poisson3d(24)
    nagg, rcp, rir, rval = aggregation_restriction(n, acp, air, seed=9)
    A, R = Csc(n, n, acp, air, aval), Csc(n, nagg, rcp, rir, rval)
    Rt = _transpose(R)
    RA = cb.LocalSpGEMMHash(PT, up(gpu_ctx, Rt), up(gpu_ctx, A))
    RAh = host(RA, nagg)
    C = cb.LocalSpGEMMHash(PT, RA, up(gpu_ctx, R))
    ORA, _, _ = oracle_spgemm(Rt, A, "plus_times", "f64")
    OC, _, _ = oracle_spgemm(ORA, R, "plus_times", "f64")
    assert_same_product(RAh, ORA, "f64", what="RtA")   # small integer sums: exact in f64
    assert_same_product(host(C, nagg), OC, "f64", what="RtAR")


def _random_symmetric(n, density, seed):
    import scipy.sparse as sp
    M = sp.random(n, n, density=density, format="csr", random_state=np.random.default_rng(seed))
    M = ((M + M.T) > 0).astype(np.float64).tocsc()
    M.setdiag(0)
    M.eliminate_zeros()
    M.sort_indices()
    return Csc(n, n, M.indptr, M.indices, M.data)


@pytest.mark.parametrize("kind,seed", [("poisson24", 1), ("poisson24", 9), ("random", 3), ("isolated", 5)])
def test_restriction_matches_host(gpu_ctx, kind, seed):
    """cbg_mis2_restriction (device MIS-2 + aggregation, RestrictionOp.h:116-290) equals the host
    restatement (inputs.aggregation_restriction) exactly: same roots, same aggregates, same R; RT = R^T."""
    if kind == "poisson24":
        n, cp, ir, val = poisson3d(24)
        G = Csc(n, n, cp, ir, val)
    elif kind == "random":
        G = _random_symmetric(6000, 6e-4, seed)
    else:   # isolated vertices (empty columns) each become their own aggregate
        G = _random_symmetric(3000, 1e-4, seed)
    nagg, rcp, rir, rval = aggregation_restriction(G.nrow, G.cp, G.ir, seed=seed)
    R, RT = cb.MIS2Restriction(up(gpu_ctx, G), seed=seed)
    Rh = host(R, G.nrow)
    assert R.getncol() == nagg
    assert np.array_equal(Rh.cp, rcp) and np.array_equal(Rh.ir, rir) and np.array_equal(Rh.val, rval)
    RTh = host(RT, nagg)
    T = _transpose(Csc(G.nrow, nagg, rcp, rir, rval))
    assert np.array_equal(RTh.cp, T.cp) and np.array_equal(RTh.ir, T.ir) and np.array_equal(RTh.val, T.val)


def test_galerkin_rap_fused_matches_reference(gpu_ctx):
    """The fused one-pass R^T A R equals the reference's two-product output (golden/galerkin.npz)."""
    z = load_fixture("galerkin")
    n, nagg = (int(x) for x in z["R_shape"])
    A = Csc(n, n, z["A_cp"], z["A_ir"], z["A_val"])
    R = Csc(n, nagg, z["R_cp"], z["R_ir"], z["R_val"])
    C = cb.GalerkinRAP(up(gpu_ctx, A), up(gpu_ctx, R))
    assert C.multiplies == A.nnz
    assert_same_product(host(C, nagg), Csc(nagg, nagg, z["C_cp"], z["C_ir"], z["C_val"]), "f64", what="fused RtAR")


@pytest.mark.parametrize("k,seed", [(24, 9), (40, 2)])
def test_galerkin_rap_fused_vs_two_products(gpu_ctx, k, seed):
    """Device R, then the fused product against the two device SpGEMMs and the oracle's two products
    (f64 within 1e-12 of sum|r a r|; weighted R rows exercise the value scaling)."""
    n, acp, air, aval = poisson3d(k)
    dA = up(gpu_ctx, Csc(n, n, acp, air, aval))
    R, RT = cb.MIS2Restriction(dA, seed=seed)
    Rh = host(R, n)
    nagg = R.getncol()
    w = 0.5 + (np.arange(Rh.nnz) % 7) / 8.0           # a weighted aggregation (one nonzero per row)
    Rw = Csc(n, nagg, Rh.cp, Rh.ir, w)
    for Rc in (Rh, Rw):
        dR = up(gpu_ctx, Rc)
        C = cb.GalerkinRAP(dA, dR)
        Rt = _transpose(Rc)
        two = cb.LocalSpGEMMHash(PT, cb.LocalSpGEMMHash(PT, up(gpu_ctx, Rt), dA), dR)
        ORA, _, _ = oracle_spgemm(Rt, Csc(n, n, acp, air, aval), "plus_times", "f64")
        OC, _, _ = oracle_spgemm(ORA, Rc, "plus_times", "f64")
        assert_same_product(host(C, nagg), OC, "f64", what="fused vs oracle")
        assert_same_product(host(C, nagg), host(two, nagg), "f64", what="fused vs two products")


def test_galerkin_rap_non_aggregation_takes_two_products(gpu_ctx):
    """An R that is no aggregation (row 0 in two aggregates): the fused kernel declines (CBG_EUNSUP, checked
    through the raw ABI) and GalerkinRAP runs the reference's two products with R^T made by cbg_transpose."""
    import ctypes
    from combblas_amd import _abi
    n = 50
    A = Csc(n, n, np.arange(n + 1), np.arange(n), np.ones(n))
    R = Csc(n, 2, np.array([0, 26, 51]), np.r_[np.arange(26), 0, np.arange(26, 50)], np.ones(51))
    dA, dR = up(gpu_ctx, A), up(gpu_ctx, R)
    res = _abi.CscResult()
    st = gpu_ctx._lib.cbg_galerkin_rap(gpu_ctx._ptr, ctypes.byref(dA._view()), ctypes.byref(dR._view()),
                                       ctypes.byref(res))
    assert st == _abi.EUNSUP
    C = cb.GalerkinRAP(dA, dR)
    ORA, _, _ = oracle_spgemm(_transpose(R), A, "plus_times", "f64")
    OC, _, _ = oracle_spgemm(ORA, R, "plus_times", "f64")
    assert_same_product(host(C, 2), OC, "f64", what="two-product RtAR")


def test_galerkin_rap_large_aggregate_falls_back(gpu_ctx):
    """An aggregate gathering more than 512 entries of A: the fused kernel declines (CBG_EUNSUP) and
    GalerkinRAP runs the reference's two products (R^T given, or built by cbg_transpose)."""
    G = _random_symmetric(400, 0.02, 4)
    n = G.nrow
    A = Csc(n, n, G.cp, G.ir, np.linspace(0.5, 1.5, G.nnz))
    agg = np.r_[np.zeros(300, np.int64), 1 + np.arange(100) % 7]     # aggregate 0 holds 300 vertices
    import scipy.sparse as sp
    Rs = sp.csc_matrix((np.ones(n), (np.arange(n), agg)), shape=(n, 8))
    Rs.sort_indices()
    R = Csc(n, 8, Rs.indptr, Rs.indices, Rs.data)
    dA, dR, dRT = up(gpu_ctx, A), up(gpu_ctx, R), up(gpu_ctx, _transpose(R))
    Rt = _transpose(R)
    ORA, _, _ = oracle_spgemm(Rt, A, "plus_times", "f64")
    OC, _, _ = oracle_spgemm(ORA, R, "plus_times", "f64")
    for C in (cb.GalerkinRAP(dA, dR, dRT), cb.GalerkinRAP(dA, dR)):   # given R^T, and R^T built on the device
        assert_same_product(host(C, 8), OC, "f64", what="fallback RtAR")


def test_galerkin_rap_big_aggregates_stay_fused(gpu_ctx):
    """Aggregates gathering 513..2048 entries of A take the fused kernel's second pass (2048-entry LDS sort)
    instead of the two-product fallback: C.multiplies = nnz(A), same product as the two products."""
    G = _random_symmetric(600, 0.02, 6)
    n = G.nrow
    A = Csc(n, n, G.cp, G.ir, np.linspace(0.5, 1.5, G.nnz))
    agg = np.r_[np.zeros(60, np.int64), np.ones(50, np.int64), 2 + np.arange(490) % 40]   # ~1400 and ~1200 entries
    import scipy.sparse as sp
    Rs = sp.csc_matrix((np.linspace(0.5, 2.0, n), (np.arange(n), agg)), shape=(n, 42))
    Rs.sort_indices()
    R = Csc(n, 42, Rs.indptr, Rs.indices, Rs.data)
    sizes = np.bincount(agg, weights=np.diff(G.cp))
    assert sizes.max() > 512 and sizes.max() <= 2048, sizes.max()
    C = cb.GalerkinRAP(up(gpu_ctx, A), up(gpu_ctx, R))
    assert C.multiplies == A.nnz   # the fused pass ran
    Rt = _transpose(R)
    ORA, _, _ = oracle_spgemm(Rt, A, "plus_times", "f64")
    OC, _, _ = oracle_spgemm(ORA, R, "plus_times", "f64")
    assert_same_product(host(C, 42), OC, "f64", what="fused RtAR, big aggregates")


# ------------------------------------------------------------------ the reference's RestrictionOp (f3)
RESTRICTION_CASES = ["poisson6", "poisson12", "poisson80", "g500_s10", "unsym700"]


def _restriction_input(z, name):
    if name.startswith("poisson"):
        n, cp, ir, val = poisson3d(int(name[len("poisson"):]))
        return Csc(n, n, cp, ir, val)
    n = len(z[f"{name}_agg"])
    cp, ir = z[f"{name}_cp"], z[f"{name}_ir"]
    return Csc(n, n, cp, ir, np.ones(len(ir)))


@pytest.mark.parametrize("name", RESTRICTION_CASES)
def test_restriction_op_matches_reference(gpu_ctx, name):
    """cbg_restriction_op on the device = the reference's RestrictionOp (3DSpGEMM/RestrictionOp.h:196-291, run by
    oracle/_ref/refrestrict at one rank, DETERMINISTIC seeds) entry for entry: the same MIS-2 set from the same
    MTRand stream, the same Select2ndRandSR aggregation, the same RandPerm column order; RT = R^T.  Poisson
    k = 6/12/80 (k = 80: 46343 aggregates, libstdc++'s one-swap-per-draw shuffle branch), the Graph500 s10
    matrix (loops, unsymmetric) and an unsymmetric matrix with isolated vertices."""
    z = load_fixture("restriction")
    G = _restriction_input(z, name)
    R, RT = cb.RestrictionOp(up(gpu_ctx, G))
    nagg = int(z[f"{name}_nagg"])
    assert R.getncol() == nagg and R.getnrow() == G.nrow
    Rh = host(R, G.nrow)
    agg = z[f"{name}_agg"].astype(np.int64)
    order = np.lexsort((np.arange(G.nrow), agg))
    cp = np.zeros(nagg + 1, np.int64)
    np.cumsum(np.bincount(agg, minlength=nagg), out=cp[1:])
    assert np.array_equal(Rh.cp, cp) and np.array_equal(Rh.ir, order) and np.all(Rh.val == 1.0)
    RTh = host(RT, nagg)
    T = _transpose(Rh)
    assert np.array_equal(RTh.cp, T.cp) and np.array_equal(RTh.ir, T.ir) and np.array_equal(RTh.val, T.val)


def test_restriction_op_seeds_change_the_aggregation(gpu_ctx):
    """Other seeds give another (still valid) aggregation: one entry per row, every aggregate non-empty."""
    n, cp, ir, val = poisson3d(12)
    dA = up(gpu_ctx, Csc(n, n, cp, ir, val))
    R1, _ = cb.RestrictionOp(dA)
    R2, _ = cb.RestrictionOp(dA, mt_seed=7, perm_seed=11)
    a, b = host(R1, n), host(R2, n)
    assert b.nnz == n and np.all(np.diff(b.cp) > 0)
    assert not (np.array_equal(a.cp, b.cp) and np.array_equal(a.ir, b.ir))


@pytest.mark.parametrize("fused", [True, False])
def test_galerkin_on_device_reference_restriction(gpu_ctx, fused):
    """End to end on the device: R from cbg_restriction_op, then R^T A R (fused, or the reference's two products
    with R^T built by cbg_transpose) equals the reference's R^T A R on the reference's R (golden/galerkin.npz,
    made by refrestrict + refprobe's LocalSpGEMMHash)."""
    z = load_fixture("galerkin")
    n, nagg = (int(x) for x in z["R_shape"])
    A = Csc(n, n, z["A_cp"], z["A_ir"], z["A_val"])
    dA = up(gpu_ctx, A)
    R, RT = cb.RestrictionOp(dA)
    Rh = host(R, n)
    assert np.array_equal(Rh.cp, z["R_cp"]) and np.array_equal(Rh.ir, z["R_ir"])
    C = cb.GalerkinRAP(dA, R, fused=fused)
    assert_same_product(host(C, nagg), Csc(nagg, nagg, z["C_cp"], z["C_ir"], z["C_val"]), "f64", what="RtAR")


def test_transpose_matches_scipy(gpu_ctx):
    M = _random_symmetric(900, 3e-3, 21)
    import scipy.sparse as sp
    S = sp.random(700, 900, density=0.01, format="csc", random_state=np.random.default_rng(5))
    S.sort_indices()
    A = Csc(700, 900, S.indptr, S.indices, S.data)
    T = cb.Transpose(up(gpu_ctx, A))
    Th = host(T, 700)
    E = S.T.tocsc()
    E.sort_indices()
    assert T.getnrow() == 900 and T.getncol() == 700
    assert np.array_equal(Th.cp, E.indptr) and np.array_equal(Th.ir, E.indices) and np.array_equal(Th.val, E.data)
    assert M.nnz > 0
