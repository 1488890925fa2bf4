"""Pins the CPU restatement (oracle/oracle.c) against outputs of the reference itself.

Fixtures come from tests/golden/make_golden.py, i.e. the reference's LocalSpGEMMHash /
LocalSpGEMM / LocalHybridSpGEMM / Mult_AnXBn_Synch (oracle/_ref/refprobe) and the MATLAB golden
3DSpGEMM/matlab/C.mtx.  If this file passes, the oracle is a trustworthy checker for the GPU path.
"""
import os

import numpy as np
import pytest

from helpers import (abs_product_sums, assert_same_product, canonical_sha256, fixture_inputs,
                     fixture_product, load_fixture, oracle_spgemm, oracle_merge, sorted_dedup_ok, Csc)

FULL = [("bcsstk01", "pt_f64_hash"), ("bcsstk01", "pt_f64_heap"), ("bcsstk01", "pt_f64_hybrid"),
        ("hepth", "pt_f64_hash"), ("largeseq", "pt_f64_hash"), ("largeseq", "mp_f64_hash"),
        ("pow2", "pt_f64_hash"), ("rect", "pt_f64_hash")] + \
       [("g500_s10", t) for t in ("pt_f64_hash", "pt_f64_heap", "pt_i64_hash", "mp_i64_hash",
                                  "s2_i64_hash", "sm_i64_hash", "smb_i64_hash")]
HASHED = [("g500_s12", t) for t in ("pt_f64_hash", "pt_f64_heap", "pt_i64_hash", "mp_i64_hash",
                                    "s2_i64_hash", "sm_i64_hash", "smb_i64_hash")]


@pytest.mark.parametrize("name,tag", FULL)
def test_oracle_matches_reference_full(name, tag):
    z = load_fixture(name)
    A, B, sr, dt = fixture_inputs(z, tag)
    C, mults, rc = oracle_spgemm(A, B, sr, dt)
    assert rc == 0
    R = fixture_product(z, tag)
    assert mults == int(z[f"C_{tag}_flops"])
    assert sorted_dedup_ok(C)
    scale = None
    if dt == "f64" and sr == "plus_times":
        scale = np.asarray(abs_product_sums(A, B)[C.ir, np.repeat(np.arange(C.ncol), np.diff(C.cp))]).ravel()
    assert_same_product(C, R, dt, scale=scale, what=f"{name}/{tag}")


@pytest.mark.parametrize("name,tag", HASHED)
def test_oracle_matches_reference_hash(name, tag):
    z = load_fixture(name)
    A, B, sr, dt = fixture_inputs(z, tag)
    C, mults, rc = oracle_spgemm(A, B, sr, dt)
    assert rc == 0
    assert mults == int(z[f"C_{tag}_flops"])
    assert C.nnz == int(z[f"C_{tag}_nnz"])
    # R-MAT values are integer multiplicities -> PlusTimes<double> is exact
    assert canonical_sha256(C.cp, C.ir, C.val) == str(z[f"C_{tag}_sha256"])


def test_matlab_golden_bcsstk01():
    """3DSpGEMM/matlab/C.mtx = MATLAB bcsstk01*bcsstk01 (multwrite.m)."""
    z = load_fixture("bcsstk01")
    A, B, sr, dt = fixture_inputs(z, "pt_f64_hash")
    C, _, rc = oracle_spgemm(A, B, sr, dt)
    assert rc == 0
    M = Csc(48, 48, z["M_matlab_cp"], z["M_matlab_ir"], z["M_matlab_val"])
    # MATLAB wrote 670 lower-triangle entries with %g-ish precision; the reference's own test
    # (test_mpipspgemm) uses EPSILON=0.01 relative (SpDefs.h:64).  Structure must be exact.
    assert np.array_equal(C.cp, M.cp) and np.array_equal(C.ir, M.ir)
    rel = np.abs(C.val - M.val) / np.maximum(np.abs(M.val), 1e-300)
    assert rel.max() < 1e-6


def test_synch_equals_local_at_one_rank():
    z = load_fixture("bcsstk01")
    R = fixture_product(z, "pt_f64_synch")
    H = fixture_product(z, "pt_f64_hash")
    assert np.array_equal(R.cp, H.cp) and np.array_equal(R.ir, H.ir)
    assert np.allclose(R.val, H.val, rtol=1e-12, atol=0)


def test_oracle_merge_equals_sum_of_parts():
    """MultiwayMerge semantics: merging C1=A*B1-split partials equals the full product."""
    z = load_fixture("g500_s10")
    A, B, sr, dt = fixture_inputs(z, "pt_i64_hash")
    # split the inner dimension k in two halves (what a 1x1x2 layout does)
    n = A.ncol
    h = n // 2
    As = A.to_scipy().tocsc()
    Bs = B.to_scipy().tocsc()
    parts = []
    for lo, hi in ((0, h), (h, n)):
        Ah = As[:, lo:hi].tocsc()
        Bh = Bs[lo:hi, :].tocsc()
        Ah.sort_indices(); Bh.sort_indices()
        Pa = Csc(Ah.shape[0], Ah.shape[1], Ah.indptr, Ah.indices, Ah.data.astype(np.int64))
        Pb = Csc(Bh.shape[0], Bh.shape[1], Bh.indptr, Bh.indices, Bh.data.astype(np.int64))
        P, _, rc = oracle_spgemm(Pa, Pb, sr, dt)
        assert rc == 0
        parts.append(P)
    M, rc = oracle_merge(parts, sr, dt)
    assert rc == 0
    R = fixture_product(z, "pt_i64_hash")
    assert_same_product(M, R, dt, what="merge")


def test_oracle_empty_and_dimension_errors():
    A = Csc(4, 3, np.zeros(4, np.int64), np.zeros(0, np.int32), np.zeros(0))
    B = Csc(3, 5, np.zeros(6, np.int64), np.zeros(0, np.int32), np.zeros(0))
    C, mults, rc = oracle_spgemm(A, B, "plus_times", "f64")
    assert rc == 0 and C.nnz == 0 and mults == 0 and len(C.cp) == 6
    Bbad = Csc(4, 5, np.zeros(6, np.int64), np.zeros(0, np.int32), np.zeros(0))
    _, _, rc = oracle_spgemm(A, Bbad, "plus_times", "f64")
    assert rc == 3002


def test_oracle_boolcopy_add_is_error():
    # two contributions to C(0,0) -> BoolCopy2nd add() would throw in the reference
    A = Csc(1, 2, [0, 1, 2], [0, 0], None)
    B = Csc(2, 1, [0, 2], [0, 1], np.array([3, 4], np.int64))
    _, _, rc = oracle_spgemm(A, B, "bool_copy2nd", "i64")
    assert rc == 13
    B1 = Csc(2, 1, [0, 1], [1], np.array([4], np.int64))
    C, _, rc = oracle_spgemm(A, B1, "bool_copy2nd", "i64")
    assert rc == 0 and C.val.tolist() == [4]


MERGE_SETS = [("split", "select2nd_i64"), ("split", "plus_times_i64"), ("rand", "select2nd_i64"),
              ("rand", "plus_times_i64"), ("rand", "min_plus_i64")]


def merge_lists(z, which):
    m, n = (int(x) for x in z[f"{which}_shape"])
    return [Csc(m, n, z[f"{which}_L{l}_cp"], z[f"{which}_L{l}_ir"], z[f"{which}_L{l}_val"])
            for l in range(int(z[f"{which}_k"]))]


@pytest.mark.parametrize("which,sr", MERGE_SETS)
def test_oracle_merge_matches_reference_multiwaymergehash(which, sr):
    """The oracle's multi-list merge equals the reference's MultiwayMergeHash (first list wins for
    Select2nd, MultiwayMerge.h:357) on reference-made partials; the heap MultiwayMerge agrees on every
    semiring except Select2nd, whose heap-pop order keeps a later list's value."""
    z = load_fixture("merge")
    lists = merge_lists(z, which)
    s, dt = sr.rsplit("_", 1)
    R, rc = oracle_merge(lists, s, dt)
    assert rc == 0
    H = Csc(0, len(z[f"{which}_{sr}_hash_cp"]) - 1, z[f"{which}_{sr}_hash_cp"], z[f"{which}_{sr}_hash_ir"],
            z[f"{which}_{sr}_hash_val"])
    assert np.array_equal(R.cp, H.cp) and np.array_equal(R.ir, H.ir) and np.array_equal(R.val, H.val)
    heap_same = np.array_equal(z[f"{which}_{sr}_heap_val"], H.val)
    assert heap_same == (s != "select2nd")


def test_merged_split_products_equal_the_product_select2nd():
    """Merging the inner-dimension split products in part order reproduces the 1-rank Select2nd
    product (min-k rule): the reference's MultiwayMergeHash output equals LocalSpGEMMHash's."""
    z = load_fixture("merge")
    f = load_fixture("g500_s10")
    assert np.array_equal(z["split_select2nd_i64_hash_cp"], f["C_s2_i64_hash_cp"])
    assert np.array_equal(z["split_select2nd_i64_hash_ir"], f["C_s2_i64_hash_ir"])
    assert np.array_equal(z["split_select2nd_i64_hash_val"], f["C_s2_i64_hash_val"])


def test_refbench_times_the_reference_on_the_bench_sample():
    """bench.py's cpu_baseline runs the reference's own LocalSpGEMMHash and 1-rank Mult_AnXBn_Synch
    (oracle/_ref/refbench) on every s-th column of B and compares their output checksum with the GPU product's
    sampled columns: here the same checksum of the oracle's product must match on the G500 s12 fixture."""
    import bench
    if not os.path.exists(bench.REFBENCH):
        pytest.skip("oracle/_ref/refbench not built (needs the reference sources)")
    z = load_fixture("g500_s12")
    A, _, _, _ = fixture_inputs(z, "pt_f64_hash")
    stride = 3
    ref = bench.reference_baseline(A.ncol, A.cp, A.ir, A.val, stride, 4, synch_factor=2)
    assert ref is not None and set(ref) == {"LocalSpGEMMHash", "Mult_AnXBn_Synch"}
    for call, s in (("LocalSpGEMMHash", stride), ("Mult_AnXBn_Synch", 2 * stride)):
        cols = np.arange(0, A.ncol, s)
        idx = np.concatenate([np.arange(A.cp[c], A.cp[c + 1]) for c in cols])
        B = Csc(A.nrow, len(cols), np.concatenate([[0], np.cumsum(np.diff(A.cp)[cols])]), A.ir[idx], A.val[idx])
        C, mults, rc = oracle_spgemm(A, B, "plus_times", "f64")
        assert rc == 0
        r = ref[call]
        assert (r["multiplies"], r["nnzC"], r["mpi_ranks"]) == (mults, C.nnz, 1), call
        assert r["checksum"] == bench.entry_checksum(C.cp, C.ir, C.val), call
