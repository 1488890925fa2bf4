"""GPU parity: libcbgpu.so (via the C ABI) against the reference fixtures and the oracle.

Bars: structure exact; integer/bool semirings bit-exact; PlusTimes<double> within
1e-12 relative (|c - r| <= 1e-12 * max(|r|, sum|a*b|)); R-MAT multiplicity values are exact.
"""
import zlib

import numpy as np
import pytest

import combblas_amd as cb
from helpers import (Csc, abs_product_sums, assert_same_product, canonical_sha256, fixture_inputs,
                     fixture_product, load_fixture, oracle_spgemm, sorted_dedup_ok)

pytestmark = pytest.mark.gpu

SRCLS = {"plus_times": cb.PlusTimesSRing, "min_plus": cb.MinPlusSRing, "select2nd": cb.Select2ndSRing,
         "select_max": cb.SelectMaxSRing, "select_max_bool": cb.SelectMaxBoolSRing,
         "bool_copy1st": cb.BoolCopy1stSRing, "bool_copy2nd": cb.BoolCopy2ndSRing}


def upload(ctx, M, dtype=None):
    return cb.SpDCCols.from_csc(ctx, M.nrow, M.ncol, M.cp, M.ir, M.val, dtype=dtype)


def gpu_product(ctx, A, B, sr, dt, sort=True):
    dA, dB = upload(ctx, A), upload(ctx, B)
    C = cb.LocalSpGEMMHash(SRCLS[sr](dt), dA, dB, sort=sort)
    cp, ir, val = C.to_host()
    return Csc(A.nrow, B.ncol, cp, ir, val), C.multiplies


def f64_scale(A, B, C):
    S = abs_product_sums(A, B)
    cols = np.repeat(np.arange(C.ncol), np.diff(C.cp))
    return np.asarray(S[C.ir, cols]).ravel()


FULL = [("bcsstk01", "pt_f64_hash"), ("hepth", "pt_f64_hash"), ("largeseq", "pt_f64_hash"),
        ("largeseq", "mp_f64_hash"), ("pow2", "pt_f64_hash"), ("rect", "pt_f64_hash")] + \
       [("g500_s10", t) for t in ("pt_f64_hash", "pt_i64_hash", "mp_i64_hash", "s2_i64_hash",
                                  "sm_i64_hash", "smb_i64_hash")]
HASHED = [("g500_s12", t) for t in ("pt_f64_hash", "pt_i64_hash", "mp_i64_hash", "s2_i64_hash",
                                    "sm_i64_hash", "smb_i64_hash")]


@pytest.mark.parametrize("name,tag", FULL)
def test_gpu_matches_reference_fixture(gpu_ctx, name, tag):
    z = load_fixture(name)
    A, B, sr, dt = fixture_inputs(z, tag)
    C, mults = gpu_product(gpu_ctx, A, B, sr, dt)
    assert mults == int(z[f"C_{tag}_flops"])
    R = fixture_product(z, tag)
    scale = f64_scale(A, B, R) if (dt == "f64" and sr == "plus_times") else None
    assert_same_product(C, R, dt, scale=scale, what=f"{name}/{tag}")


@pytest.mark.parametrize("name,tag", HASHED)
def test_gpu_matches_reference_hash(gpu_ctx, name, tag):
    z = load_fixture(name)
    A, B, sr, dt = fixture_inputs(z, tag)
    C, mults = gpu_product(gpu_ctx, A, B, sr, dt)
    assert mults == int(z[f"C_{tag}_flops"])
    assert C.nnz == int(z[f"C_{tag}_nnz"])
    assert canonical_sha256(C.cp, C.ir, C.val) == str(z[f"C_{tag}_sha256"])


def test_matlab_golden(gpu_ctx):
    z = load_fixture("bcsstk01")
    A, B, sr, dt = fixture_inputs(z, "pt_f64_hash")
    C, _ = gpu_product(gpu_ctx, A, B, sr, dt)
    assert np.array_equal(C.cp, z["M_matlab_cp"]) and np.array_equal(C.ir, z["M_matlab_ir"])
    M = z["M_matlab_val"]
    assert np.max(np.abs(C.val - M) / np.abs(M)) < 1e-6


# ------------------------------------------------------------------ random cases vs the oracle
def rand_csc(rng, m, n, density, dtype, pattern=False, lo=-5, hi=6):
    import scipy.sparse as sp
    S = sp.random(m, n, density=density, format="csc", random_state=rng,
                  data_rvs=lambda k: np.ones(k)).astype(np.float64)
    S.sort_indices()
    nnz = S.nnz
    if pattern:
        val = None
    elif dtype in ("f64", "f32"):
        val = rng.uniform(-2, 2, nnz).astype(np.float64 if dtype == "f64" else np.float32)
    elif dtype == "bool":
        val = np.ones(nnz, np.uint8)
    else:
        val = rng.integers(lo, hi, nnz).astype(np.int64 if dtype == "i64" else np.int32)
    return Csc(m, n, S.indptr, S.indices, val)


CASES = [("plus_times", "f64"), ("plus_times", "f32"), ("plus_times", "i64"), ("plus_times", "i32"),
         ("plus_times", "bool"), ("min_plus", "f64"), ("min_plus", "i64"), ("min_plus", "i32"),
         ("select2nd", "i64"), ("select2nd", "f64"), ("select_max", "i64"), ("select_max", "f64"),
         ("select_max_bool", "i64")]


@pytest.mark.parametrize("sr,dt", CASES)
@pytest.mark.parametrize("shape", [(50, 40, 60, 0.05), (300, 200, 250, 0.02), (2000, 1500, 1800, 0.004)])
def test_gpu_random_vs_oracle(gpu_ctx, sr, dt, shape):
    m, k, n, d = shape
    rng = np.random.default_rng(zlib.crc32(repr((sr, dt, shape)).encode()))   # stable across processes
    A = rand_csc(rng, m, k, d, dt, pattern=(sr == "select_max_bool"))
    B = rand_csc(rng, k, n, d, dt)
    R, rmults, rc = oracle_spgemm(A, B, sr, dt)
    assert rc == 0
    C, mults = gpu_product(gpu_ctx, A, B, sr, dt)
    assert mults == rmults
    assert sorted_dedup_ok(C)
    if dt == "f32":
        assert_same_product(C, R, dt, rtol=1e-5, scale=f64_scale(A, B, R), what=f"{sr}/{dt}")
    else:
        scale = f64_scale(A, B, R) if dt == "f64" and sr == "plus_times" else None
        assert_same_product(C, R, dt, scale=scale, what=f"{sr}/{dt}")


def test_gpu_min_plus_infinity(gpu_ctx):
    """inf_plus: max() is infinity and absorbs (Semirings.h:40-47)."""
    big = np.iinfo(np.int64).max
    A = Csc(3, 2, [0, 2, 3], [0, 2, 1], np.array([big, 5, 7], np.int64))
    B = Csc(2, 2, [0, 2, 3], [0, 1, 1], np.array([1, big, 2], np.int64))
    R, _, rc = oracle_spgemm(A, B, "min_plus", "i64")
    C, _ = gpu_product(gpu_ctx, A, B, "min_plus", "i64")
    assert_same_product(C, R, "i64")


def test_gpu_boolcopy(gpu_ctx):
    A = Csc(3, 2, [0, 1, 2], [0, 2], None)
    B = Csc(2, 2, [0, 1, 2], [1, 0], np.array([3.5, 4.5]))
    C, _ = gpu_product(gpu_ctx, A, B, "bool_copy2nd", "f64")
    assert C.ir.tolist() == [2, 0] and C.val.tolist() == [3.5, 4.5]
    Bdup = Csc(2, 1, [0, 2], [0, 1], np.array([3.0, 4.0]))
    Adup = Csc(1, 2, [0, 1, 2], [0, 0], None)
    with pytest.raises(cb.CbgError) as ei:
        gpu_product(gpu_ctx, Adup, Bdup, "bool_copy2nd", "f64")
    assert ei.value.status == 13


def test_gpu_empty_and_dim_errors(gpu_ctx):
    A = Csc(4, 3, np.zeros(4, np.int64), np.zeros(0, np.int32), np.zeros(0))
    B = Csc(3, 5, [0, 1, 1, 1, 1, 1], [2], np.ones(1))
    C, m = gpu_product(gpu_ctx, A, B, "plus_times", "f64")
    assert C.nnz == 0 and m == 0 and len(C.cp) == 6
    Bbad = Csc(4, 5, np.zeros(6, np.int64), np.zeros(0, np.int32), np.zeros(0))
    with pytest.raises(cb.CbgError) as ei:
        gpu_product(gpu_ctx, A, Bbad, "plus_times", "f64")
    assert ei.value.status == 3002


def _check_vs_oracle(ctx, A, B, sr="plus_times", dt="f64"):
    R, rm, rc = oracle_spgemm(A, B, sr, dt)
    assert rc == 0
    C, m = gpu_product(ctx, A, B, sr, dt)
    assert m == rm
    assert_same_product(C, R, dt, scale=f64_scale(A, B, R) if dt == "f64" else None)
    return C


def test_gpu_hash_overflow_fallback(gpu_ctx):
    """Rows clustered at the top of a wide span defeat the order-preserving hash; the column must be
    re-done by the windowed dense kernel (fallback list), still exact."""
    n = 1 << 20
    rows = np.r_[0, np.arange(n - 3000, n)].astype(np.int32)
    A = Csc(n, 1, [0, len(rows)], rows, np.arange(1, len(rows) + 1, dtype=np.float64))
    B = Csc(1, 1, [0, 1], [0], np.array([2.0]))
    C = _check_vs_oracle(gpu_ctx, A, B)
    assert gpu_ctx.last_profile()["bins"][15] >= 1


def test_gpu_heavy_column_window_kernel(gpu_ctx):
    """One output column with ~60k entries spread over 2^21 rows -> windowed kernel, many windows,
    long segments (wavefront path) and short segments (lane path) mixed."""
    rng = np.random.default_rng(7)
    n = 1 << 21
    cols = []
    cp = [0]
    for j in range(40):
        L = int(rng.integers(1, 4000)) if j % 3 else int(rng.integers(1, 20))
        cols.append(np.sort(rng.choice(n, L, replace=False)).astype(np.int32))
        cp.append(cp[-1] + L)
    A = Csc(n, 40, cp, np.concatenate(cols), rng.uniform(-1, 1, cp[-1]))
    B = Csc(40, 3, [0, 40, 45, 60], np.r_[np.arange(40), np.arange(5), np.arange(10, 25)].astype(np.int32),
            rng.uniform(-1, 1, 60))
    _check_vs_oracle(gpu_ctx, A, B)


@pytest.mark.parametrize("n,sr,dt", [(1 << 21, "plus_times", "f64"), (3 << 19, "min_plus", "i64"),
                                      (1 << 21, "select_max", "i64"), (1 << 24, "plus_times", "i64")])
def test_gpu_wide_column_parts(gpu_ctx, n, sr, dt):
    """Wide output columns (bitmap > 16384 words): symbolic runs as (column, 2^19-row part) items with
    split-table segments for long A columns and filtered short ones; spans not aligned to parts,
    columns touching 1..all parts.  n = 2^24 puts 32 parts in one column -> windowed symbolic."""
    rng = np.random.default_rng(n % 1000 + len(sr))
    ncolA = 120
    lens = np.where(rng.random(ncolA) < 0.4, rng.integers(16, 2500, ncolA), rng.integers(1, 16, ncolA))
    cols = []
    for c, L in enumerate(lens):
        lo = int(rng.integers(0, n // 2)) if c % 4 == 0 else 0
        hi = n if c % 5 else int(rng.integers(lo + L + 1, n))
        cols.append(np.sort(lo + rng.choice(hi - lo, int(L), replace=False)).astype(np.int32))
    cp = np.r_[0, np.cumsum(lens)]
    vals = rng.integers(-4, 5, cp[-1]).astype(np.int64) if dt == "i64" else rng.uniform(-1, 1, cp[-1])
    A = Csc(n, ncolA, cp, np.concatenate(cols), vals)
    nb = 12
    bcp, bir = [0], []
    for j in range(nb):
        k = np.sort(rng.choice(ncolA, int(rng.integers(3, 60)), replace=False))
        bir.append(k.astype(np.int32))
        bcp.append(bcp[-1] + len(k))
    bv = rng.integers(-4, 5, bcp[-1]).astype(np.int64) if dt == "i64" else rng.uniform(-1, 1, bcp[-1])
    B = Csc(ncolA, nb, bcp, np.concatenate(bir), bv)
    _check_vs_oracle(gpu_ctx, A, B, sr, dt)
    assert gpu_ctx.last_profile()["bins"][12] > 0


@pytest.mark.parametrize("scale", [12, 14, 16])
def test_gpu_rmat_vs_oracle(gpu_ctx, scale):
    n, cp, ir, val = cb.generate_rmat_host(scale, 16, seed=scale)
    A = Csc(n, n, cp, ir, val)
    R, rm, rc = oracle_spgemm(A, A, "plus_times", "f64")
    C, m = gpu_product(gpu_ctx, A, A, "plus_times", "f64")
    assert m == rm
    # multiplicity values -> exact sums
    assert np.array_equal(C.cp, R.cp) and np.array_equal(C.ir, R.ir) and np.array_equal(C.val, R.val)


def test_gpu_dcsc_input_view(gpu_ctx):
    """The reference's DCSC arrays (cp[nzc+1], jc[nzc], ir, numx; int64 IT) go straight in."""
    import ctypes
    from combblas_amd import _abi
    z = load_fixture("g500_s10")
    A, B, sr, dt = fixture_inputs(z, "pt_f64_hash")
    nzc_cols = np.flatnonzero(np.diff(B.cp) > 0).astype(np.int64)
    dcp = np.r_[B.cp[nzc_cols], B.cp[-1]].astype(np.int64)
    ir64 = B.ir.astype(np.int64)
    vb = _abi.DcscView(B.nrow, B.ncol, B.nnz, len(nzc_cols), dcp.ctypes.data, nzc_cols.ctypes.data,
                       ir64.ctypes.data, 8, 8, B.val.ctypes.data, _abi.F64, 0)
    dA = upload(gpu_ctx, A)
    va = dA._view()
    res = _abi.CscResult()
    m = ctypes.c_int64()
    _abi.check(gpu_ctx._lib.cbg_spgemm_local(gpu_ctx._ptr, ctypes.byref(va), ctypes.byref(vb), 0, _abi.F64, 1,
                                             ctypes.byref(res), ctypes.byref(m)))
    C = cb.SpTuples._from_result(gpu_ctx, res)
    cp, irc, v = C.to_host()
    R = fixture_product(z, "pt_f64_hash")
    assert np.array_equal(cp, R.cp) and np.array_equal(irc, R.ir) and np.array_equal(v, R.val)


def test_gpu_unit_overflow_fallback(gpu_ctx):
    """A heavy column (nnz > 4096 -> units) whose multi-subwindow unit has its rows packed at the top:
    the unit's order-preserving hash overflows and is re-run as dense single-subwindow units."""
    W = 8192
    # 3000 rows packed under the top of the first unit's range [0, 20W): their order-preserving homes
    # sit within 150 slots of T = 8192, so linear probing runs past the table tail
    rows = np.r_[np.arange(10), np.arange(20 * W - 3000, 20 * W), 20 * W + np.arange(0, 4000, 2)].astype(np.int32)
    n = 1 << 20
    A = Csc(n, 1, [0, len(rows)], rows, np.arange(1, len(rows) + 1, dtype=np.float64))
    B = Csc(1, 1, [0, 1], [0], np.array([2.0]))
    # PlusTimes takes the rank mode (exact slots: no hash, nothing overflows)
    _check_vs_oracle(gpu_ctx, A, B)
    assert gpu_ctx.last_profile()["bins"][12] == 1          # one heavy column
    # BoolCopy semirings keep the hash mode (it detects a second contribution): overflow + dense re-run
    _check_vs_oracle(gpu_ctx, A, B, sr="bool_copy1st")
    prof = gpu_ctx.last_profile()
    assert prof["bins"][12] == 1          # one heavy column
    assert prof["bins"][14] >= 1          # at least one unit re-run densely


def test_gpu_heavy_units_many_columns(gpu_ctx):
    """Many heavy columns with mixed long/short A segments, every semiring family."""
    rng = np.random.default_rng(11)
    n = 1 << 18
    ncolA = 300
    lens = np.where(rng.random(ncolA) < 0.3, rng.integers(64, 3000, ncolA), rng.integers(1, 40, ncolA))
    cols = [np.sort(rng.choice(n, L, replace=False)).astype(np.int32) for L in lens]
    cp = np.r_[0, np.cumsum(lens)]
    A = Csc(n, ncolA, cp, np.concatenate(cols), rng.integers(-3, 4, cp[-1]).astype(np.int64))
    nb = 20
    bcp = [0]
    bir = []
    for j in range(nb):
        k = np.sort(rng.choice(ncolA, int(rng.integers(5, 120)), replace=False))
        bir.append(k.astype(np.int32))
        bcp.append(bcp[-1] + len(k))
    B = Csc(ncolA, nb, bcp, np.concatenate(bir), rng.integers(-3, 4, bcp[-1]).astype(np.int64))
    for sr in ("plus_times", "min_plus", "select2nd", "select_max"):
        _check_vs_oracle(gpu_ctx, A, B, sr, "i64")
    assert gpu_ctx.last_profile()["bins"][12] > 0


@pytest.mark.parametrize("sr,dt", [("plus_times", "f64"), ("min_plus", "i64"), ("select2nd", "i64"),
                                   ("select_max", "i64"), ("bool_copy2nd", "f64"), ("plus_times", "f32"),
                                   ("plus_times", "i32"), ("min_plus", "i32")])
def test_gpu_heavy_rank_mode_multichunk(gpu_ctx, sr, dt):
    """Heavy columns whose B column holds > 1024 nonzeros (the rank mode streams the unit's segments
    twice: mark pass, accumulate pass), spans below and above the rank-mode limit, plus a column
    whose units are single-chunk.  BoolCopy2nd keeps the hash mode (A columns have disjoint rows,
    so no output gets a second contribution)."""
    rng = np.random.default_rng(23)
    n = 1 << 20
    ncolA = 6000
    if sr == "bool_copy2nd":   # disjoint rows per A column -> each output has exactly one product
        perm = rng.permutation(n)[: ncolA * 2]
        cols = [np.sort(perm[2 * k: 2 * k + 2]).astype(np.int32) for k in range(ncolA)]
    else:
        hi = np.where(np.arange(ncolA) < 3000, 300_000, n)   # first half: narrow span, second: full
        cols = [np.sort(rng.choice(int(hi[k]), int(rng.integers(1, 6)), replace=False)).astype(np.int32)
                for k in range(ncolA)]
    cp = np.r_[0, np.cumsum([len(c) for c in cols])]
    npdt = {"f64": np.float64, "f32": np.float32, "i64": np.int64, "i32": np.int32}[dt]
    A = Csc(n, ncolA, cp, np.concatenate(cols), rng.integers(1, 9, cp[-1]).astype(npdt))
    pick = [np.arange(0, 3000, dtype=np.int32),                      # nb = 3000, span <= 300k rows
            np.arange(3000, 6000, 2, dtype=np.int32),                # nb = 1500, full span
            np.sort(rng.choice(3000, 900, replace=False)).astype(np.int32)]   # single chunk
    bcp = np.r_[0, np.cumsum([len(x) for x in pick])]
    B = Csc(ncolA, len(pick), bcp, np.concatenate(pick), rng.integers(1, 9, bcp[-1]).astype(npdt))
    _check_vs_oracle(gpu_ctx, A, B, sr, dt)
    prof = gpu_ctx.last_profile()
    assert prof["bins"][12] >= 1   # heavy columns present
    if sr != "bool_copy2nd":       # rank mode: units are sized per accumulator width, none re-run
        assert prof["bins"][14] == 0


@pytest.mark.parametrize("sr,dt", [("plus_times", "f64"), ("plus_times", "i64"), ("min_plus", "i64"),
                                   ("select2nd", "i64"), ("select_max", "f64")])
@pytest.mark.parametrize("nparts", [1, 2, 4])
def test_gpu_multiway_merge_vs_oracle(gpu_ctx, sr, dt, nparts):
    """MultiwayMerge (MultiwayMerge.h:411-526): k column-sorted partials -> one, duplicates via SR::add in
    list order (Select2nd: the first list holding the entry wins)."""
    from helpers import oracle_merge
    rng = np.random.default_rng(nparts * 7 + len(sr))
    parts = [rand_csc(rng, 3000, 500, 0.01 + 0.01 * p, dt) for p in range(nparts)]
    R, rc = oracle_merge(parts, sr, dt)
    assert rc == 0
    dparts = [upload(gpu_ctx, P) for P in parts]
    M = cb.MultiwayMerge(SRCLS[sr](dt), dparts)
    cp, ir, val = M.to_host()
    C = Csc(3000, 500, cp, ir, val)
    assert_same_product(C, R, dt, scale=np.abs(R.val) * nparts if dt == "f64" else None, what=f"merge {sr}")


def test_gpu_merge_of_split_products_equals_product(gpu_ctx):
    """1x1x2-style: split the inner dimension, multiply the halves on the GPU, merge on the GPU."""
    z = load_fixture("g500_s10")
    A, B, sr, dt = fixture_inputs(z, "pt_i64_hash")
    As, Bs = A.to_scipy().tocsc(), B.to_scipy().tocsc()
    h = A.ncol // 2
    halves = []
    for lo, hi in ((0, h), (h, A.ncol)):
        Ah, Bh = As[:, lo:hi].tocsc(), Bs[lo:hi, :].tocsc()
        Ah.sort_indices(); Bh.sort_indices()
        dA = cb.SpDCCols.from_csc(gpu_ctx, Ah.shape[0], Ah.shape[1], Ah.indptr, Ah.indices, Ah.data.astype(np.int64))
        dB = cb.SpDCCols.from_csc(gpu_ctx, Bh.shape[0], Bh.shape[1], Bh.indptr, Bh.indices, Bh.data.astype(np.int64))
        halves.append(cb.LocalSpGEMMHash(cb.PlusTimesSRing("i64"), dA, dB))
    M = cb.MultiwayMerge(cb.PlusTimesSRing("i64"), halves)
    cp, ir, val = M.to_host()
    R = fixture_product(z, "pt_i64_hash")
    assert np.array_equal(cp, R.cp) and np.array_equal(ir, R.ir) and np.array_equal(val, R.val)


def test_gpu_rmat_s18_sampled_vs_oracle(gpu_ctx):
    """R-MAT s18 A*A on the device (SUBW subwindows, multi-unit heavy columns, 2^18-row symbolic parts):
    every 3rd column of the full product against the oracle's product of those columns, bit-exact
    (multiplicity values), and the total multiplies against estimateFLOP by numpy."""
    n, cp, ir, val = cb.generate_rmat_host(18, 16, seed=1)
    dA = cb.SpDCCols.from_csc(gpu_ctx, n, n, cp, ir, val)
    C = cb.LocalSpGEMMHash(cb.PlusTimesSRing("f64"), dA, dA)
    alen = np.diff(cp)
    assert C.multiplies == int(alen[ir].sum())
    assert gpu_ctx.last_profile()["bins"][12] > 0
    cols = np.arange(0, n, 3)
    sel = np.concatenate([np.arange(cp[c], cp[c + 1]) for c in cols])
    B = Csc(n, len(cols), np.r_[0, np.cumsum(alen[cols])], ir[sel], val[sel])
    R, rm, rc = oracle_spgemm(Csc(n, n, cp, ir, val), B, "plus_times", "f64")
    assert rc == 0
    S = C.select_columns(cols)
    scp, sir, sval = S.to_host()
    assert np.array_equal(scp, R.cp) and np.array_equal(sir, R.ir) and np.array_equal(sval, R.val)


def test_gpu_col_select(gpu_ctx):
    """cbg_col_select: arbitrary column subsets (repeats, any order) of a device CSC."""
    rng = np.random.default_rng(3)
    M = rand_csc(rng, 400, 300, 0.03, "i64")
    d = upload(gpu_ctx, M)
    cols = np.r_[rng.integers(0, 300, 200), 7, 7, 299, 0]
    S = d.select_columns(cols)
    cp, ir, val = S.to_host()
    R = M.to_scipy()[:, cols].tocsc()
    R.sort_indices()
    assert np.array_equal(cp, R.indptr) and np.array_equal(ir, R.indices) and np.array_equal(val, R.data)
    with pytest.raises(cb.CbgError) as ei:
        d.select_columns([300])
    assert ei.value.status == 3002


def test_gpu_bpos_guard(gpu_ctx):
    """Select2nd / BoolCopy2nd accumulate an int32 B position: nnz(B) >= 2^31 is refused (CBG_EUNSUP)
    before any device work, instead of silently truncating."""
    import ctypes
    from combblas_amd import _abi
    A = upload(gpu_ctx, rand_csc(np.random.default_rng(1), 50, 40, 0.1, "i64"))
    va = A._view()
    big = (1 << 31)
    vb = _abi.DcscView(40, 10, big, 10, va.cp, None, va.ir, 4, 8, va.val, _abi.I64, 1)   # never read
    res = _abi.CscResult()
    m = ctypes.c_int64()
    for sr in (_abi.SR_SELECT2ND, _abi.SR_BOOL_COPY2ND):
        st = gpu_ctx._lib.cbg_spgemm_local(gpu_ctx._ptr, ctypes.byref(va), ctypes.byref(vb), sr, _abi.I64, 1,
                                           ctypes.byref(res), ctypes.byref(m))
        assert st == _abi.EUNSUP


@pytest.mark.parametrize("which,sr", [("split", "select2nd_i64"), ("split", "plus_times_i64"),
                                      ("rand", "select2nd_i64"), ("rand", "plus_times_i64"),
                                      ("rand", "min_plus_i64")])
def test_gpu_merge_matches_reference_multiwaymergehash(gpu_ctx, which, sr):
    """cbg_merge equals the reference's MultiwayMergeHash on reference-made lists (tests/golden/merge.npz,
    refprobe `merge`): duplicates combined in list order, Select2nd keeping the first list's value."""
    z = load_fixture("merge")
    m, n = (int(x) for x in z[f"{which}_shape"])
    lists = [upload(gpu_ctx, Csc(m, n, z[f"{which}_L{l}_cp"], z[f"{which}_L{l}_ir"], z[f"{which}_L{l}_val"]))
             for l in range(int(z[f"{which}_k"]))]
    s, dt = sr.rsplit("_", 1)
    M = cb.MultiwayMerge(SRCLS[s](dt), lists)
    cp, ir, val = M.to_host()
    assert np.array_equal(cp, z[f"{which}_{sr}_hash_cp"]) and np.array_equal(ir, z[f"{which}_{sr}_hash_ir"])
    assert np.array_equal(val, z[f"{which}_{sr}_hash_val"])


def test_gpu_two_way_merge_edge_cases(gpu_ctx):
    """The two-way merge kernel: columns longer than one 256-position window with duplicates straddling
    window ends, empty columns on either side, an unsorted partial (declined, the hash merge takes it:
    same result), and BoolCopy1st duplicates (CBG_EADD, as the reference's add() throws)."""
    from helpers import oracle_merge
    rng = np.random.default_rng(5)
    n, m = 4000, 7
    cols_a, cols_b = [], []
    for j in range(m):
        la, lb = [0, 300, 1000, 257, 0, 3000, 1][j], [0, 0, 999, 300, 5, 2999, 1][j]
        base = rng.choice(n, size=min(n, la + lb), replace=False)
        a = np.sort(base[:la]) if la else np.zeros(0, np.int64)
        # part 1 shares about half of part 0's rows (duplicate pairs), the rest fresh
        share = rng.choice(a, size=min(len(a), lb // 2), replace=False) if la else np.zeros(0, np.int64)
        b = np.unique(np.concatenate([share, base[la:la + lb - len(share)]]))[:lb]
        cols_a.append(a)
        cols_b.append(np.sort(b))

    def mk(cols):
        cp = np.concatenate([[0], np.cumsum([len(c) for c in cols])]).astype(np.int64)
        ir = np.concatenate(cols).astype(np.int32)
        return Csc(n, m, cp, ir, rng.integers(1, 9, len(ir)).astype(np.int64))
    P0, P1 = mk(cols_a), mk(cols_b)
    for sr in ("plus_times", "min_plus", "select2nd", "select_max"):
        R, rc = oracle_merge([P0, P1], sr, "i64")
        assert rc == 0
        M = cb.MultiwayMerge(SRCLS[sr]("i64"), [upload(gpu_ctx, P0), upload(gpu_ctx, P1)])
        cp, ir, val = M.to_host()
        assert_same_product(Csc(n, m, cp, ir, val), R, "i64", what=f"two-way merge {sr}")
    # unsorted part 1 (column 2 reversed): the hash merge's result, row-sorted
    ir1 = P1.ir.copy()
    ir1[P1.cp[2]:P1.cp[3]] = ir1[P1.cp[2]:P1.cp[3]][::-1]
    P1u = Csc(n, m, P1.cp, ir1, P1.val.copy())
    P1u.val[P1.cp[2]:P1.cp[3]] = P1.val[P1.cp[2]:P1.cp[3]][::-1]
    R, rc = oracle_merge([P0, P1], "plus_times", "i64")
    M = cb.MultiwayMerge(SRCLS["plus_times"]("i64"), [upload(gpu_ctx, P0), upload(gpu_ctx, P1u)])
    cp, ir, val = M.to_host()
    assert_same_product(Csc(n, m, cp, ir, val), R, "i64", what="two-way merge, unsorted part")
    with pytest.raises(cb.CbgError) as ei:
        cb.MultiwayMerge(SRCLS["bool_copy1st"]("i64"), [upload(gpu_ctx, P0), upload(gpu_ctx, P1)])
    assert ei.value.status == 13


@pytest.mark.parametrize("flat", ["1", "0"])
@pytest.mark.parametrize("sr,dt", [("plus_times", "f64"), ("plus_times", "i64"), ("min_plus", "i64"),
                                   ("select2nd", "i64"), ("select_max", "f64")])
def test_gpu_flat_merge_tiles(gpu_ctx, monkeypatch, flat, sr, dt):
    """The flat two-way merge (1023-position tiles over the whole merged sequence: count pass, scan, fill pass) and the per-column one give
    the oracle's MultiwayMerge: leading / inner / trailing runs of empty columns, a one-entry column before a
    10k-row column whose rows all pair up (every tile boundary falls inside a pair and moves back), short
    columns sharing tiles, one-sided columns, and an empty partial."""
    from helpers import oracle_merge
    monkeypatch.setenv("CBG_MERGE_FLAT", flat)
    rng = np.random.default_rng(zlib.crc32(repr((sr, dt)).encode()))
    n = 20000
    lens = [(0, 0)] * 5 + [(1, 0), (10000, 10000), (0, 0), (3, 4), (0, 7), (9, 0)] + [(0, 0)] * 300 + \
           [(int(a), int(b)) for a, b in rng.integers(0, 40, (2000, 2))] + [(2500, 1700), (1, 1)] + [(0, 0)] * 50
    cols_a, cols_b = [], []
    for j, (la, lb) in enumerate(lens):
        if j == 6:   # identical rows: every entry is a pair
            a = np.sort(rng.choice(n, la, replace=False))
            cols_a.append(a); cols_b.append(a.copy())
            continue
        base = rng.choice(n, la + lb, replace=False)
        a = np.sort(base[:la])
        share = rng.choice(a, min(la, lb // 2), replace=False) if la else np.zeros(0, np.int64)
        b = np.unique(np.concatenate([share, base[la:la + lb - len(share)]]))[:lb]
        cols_a.append(a); cols_b.append(np.sort(b))
    m = len(lens)
    npdt = np.float64 if dt == "f64" else np.int64

    def mk(cols):
        cp = np.concatenate([[0], np.cumsum([len(c) for c in cols])]).astype(np.int64)
        ir = np.concatenate(cols).astype(np.int32)
        v = rng.random(len(ir)) + 0.5 if dt == "f64" else rng.integers(1, 9, len(ir))
        return Csc(n, m, cp, ir, v.astype(npdt))
    P0, P1 = mk(cols_a), mk(cols_b)
    E = Csc(n, m, np.zeros(m + 1, np.int64), np.zeros(0, np.int32), np.zeros(0, npdt))
    for parts in ([P0, P1], [P1, P0], [P0, E], [E, P1], [E, E]):
        R, rc = oracle_merge(parts, sr, dt)
        assert rc == 0
        M = cb.MultiwayMerge(SRCLS[sr](dt), [upload(gpu_ctx, P) for P in parts])
        cp, ir, val = M.to_host()
        assert_same_product(Csc(n, m, cp, ir, val), R, dt, scale=np.abs(R.val) * 2 if dt == "f64" else None,
                            what=f"flat={flat} merge {sr}")


@pytest.mark.parametrize("dt", ["i64", "f64"])
def test_gpu_repeated_b_rows_in_wide_columns(gpu_ctx, dt):
    """B columns that name one long A column hundreds of times (repeated rows, unsorted): the wide-column symbolic
    pass (k_sym_part, 32-bit segment staging) sees chunks of 512 segments of up to 2^18 entries each -- the most a
    chunk can stage, since a segment is one A column narrowed to one part -- and the rows-known numeric units sum the
    repeats.  Bit-exact (i64) / within 1e-12 (f64) against the oracle."""
    rng = np.random.default_rng(31)
    n = 1 << 20
    lens = [200_000, 150_000, 3, 40_000, 1]
    cols = [np.sort(rng.choice(n, L, replace=False)).astype(np.int32) for L in lens]
    cp = np.r_[0, np.cumsum(lens)]
    vals = rng.integers(-3, 4, cp[-1]).astype(np.int64) if dt == "i64" else rng.uniform(-1, 1, cp[-1])
    A = Csc(n, len(lens), cp, np.concatenate(cols), vals)
    bcols = [np.r_[np.zeros(700, np.int32), [3, 2, 4]],            # 700 x column 0, then others
             rng.permutation(np.r_[np.ones(600, np.int32), np.full(300, 3, np.int32), [0]]).astype(np.int32),
             np.array([4, 4, 2, 2, 2], np.int32)]
    bcp = np.r_[0, np.cumsum([len(c) for c in bcols])]
    bv = (rng.integers(-2, 3, bcp[-1]).astype(np.int64) if dt == "i64" else rng.uniform(-1, 1, bcp[-1]))
    B = Csc(len(lens), len(bcols), bcp, np.concatenate(bcols), bv)
    _check_vs_oracle(gpu_ctx, A, B, "plus_times", dt)
    prof = gpu_ctx.last_profile()
    assert prof["bins"][12] > 0 or prof["bins"][13] > 0   # wide / heavy columns took the part and unit paths
