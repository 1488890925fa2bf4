"""GPU: the fiber exchange's wire codec (cbg_fiber_codec = grid.hip's production fiber_encode / fiber_decode) round
trips bit for bit on every wire form, the symbolic-only estimate, and the heavy-kernel counts in cbg_profile.

The codec replaces the reference's SpTuples all-to-all of the 3D fiber reduction (ParFriends.h:3119-3153); its
bar is losslessness (bit-exact round trip of colptr, rows and value bits), so there is no reference output to pin
it against beyond the product it carries (covered by test_dist_gpu.py through the real exchange)."""
import numpy as np
import pytest

import combblas_amd as cb
from helpers import Csc, oracle_spgemm

pytestmark = pytest.mark.gpu

K_HEAVY = 4096


def _mat(ctx, n, ncol, cols, dtype="f64"):
    """CSC from a list of (rows, values) per column (rows ascending)."""
    cp = np.zeros(ncol + 1, np.int64)
    ir, val = [], []
    for c, (r, v) in enumerate(cols):
        cp[c + 1] = cp[c] + len(r)
        ir.append(np.asarray(r, np.int32))
        val.append(np.asarray(v))
    ir = np.concatenate(ir) if ir else np.zeros(0, np.int32)
    val = np.concatenate(val) if val else np.zeros(0)
    return cb.SpDCCols.from_csc(ctx, n, ncol, cp, ir, val, dtype=dtype)


def _check(st, rows=None, vals=None):
    assert st["roundtrip_exact"] == 1 and st["mismatches"] == 0, st
    assert st["wire_bytes"] == (st["header_bytes"] + st["row_bytes"] + st["escape_bytes"] + st["value_bytes"]
                                + st["value_header_bytes"])
    if rows is not None:
        assert st["row_formats"] == rows, st
    if vals is not None:
        assert st["value_formats"] == vals, st


@pytest.mark.parametrize("chunks", [1, 2, 3, 8])
def test_codec_rmat_product_varint(gpu_ctx, chunks):
    """An R-MAT A*A partial (multiplicities): varint row gaps and varint integer values, every chunk exact."""
    n, cp, ir, val = cb.generate_rmat_host(14, 16, seed=5)
    A = cb.SpDCCols.from_csc(gpu_ctx, n, n, cp, ir, val)
    C = cb.LocalSpGEMMHash(cb.PlusTimesSRing("f64"), A, A)
    st = C.fiber_codec(chunks)
    _check(st, rows=1 << 2, vals=1 << 3)
    assert st["chunks"] == chunks and st["entries"] == C.getnnz()
    assert st["wire_bytes"] < 4 * C.getnnz()   # ~2-3 bytes per entry


def test_codec_forms_and_edges(gpu_ctx):
    rng = np.random.default_rng(11)
    n = 1 << 20
    # large row gaps (> 65534) force escapes in the u16 gap form; values u16 integers -> u16
    cols = [(np.sort(rng.choice(n, 50, replace=False)), rng.integers(0, 65536, 50).astype(float)) for _ in range(30)]
    cols[3] = ([], [])                         # empty column
    cols[7] = ([n - 1], [65535.0])             # a lone last row
    st = _mat(gpu_ctx, n, 30, cols).fiber_codec(2)
    _check(st)
    assert st["entries"] == sum(len(c[0]) for c in cols)
    # real values: native f64 on the wire
    cols = [(np.sort(rng.choice(4096, 200, replace=False)), rng.standard_normal(200)) for _ in range(40)]
    _check(_mat(gpu_ctx, 4096, 40, cols).fiber_codec(4), vals=1 << 0)
    # f32-exact non-integers -> f32; negative zero and signed values survive bit for bit
    cols = [(np.arange(0, 3000, 3), (rng.standard_normal(1000).astype(np.float32)).astype(float)) for _ in range(5)]
    cols[0][1][0] = -0.0
    _check(_mat(gpu_ctx, 3000, 5, cols).fiber_codec(2), vals=1 << 1)
    # integers above 2^32 -> not varint, not f32/u16: native
    cols = [([1, 2, 3], [2.0 ** 40 + 1.0, 3.0, 1.0])]
    _check(_mat(gpu_ctx, 10, 1, cols).fiber_codec(1), vals=1 << 0)
    # an f32 product and a pattern (bool) product: native values, coded rows
    cols = [(np.arange(0, 9000, 7), np.ones(1286)) for _ in range(3)]
    _check(_mat(gpu_ctx, 9000, 3, cols, dtype="f32").fiber_codec(2))
    _check(_mat(gpu_ctx, 9000, 3, cols, dtype="bool").fiber_codec(2))
    # no entries at all; more chunks than columns
    st = _mat(gpu_ctx, 100, 4, [([], [])] * 4).fiber_codec(8)
    _check(st)
    assert st["entries"] == 0 and st["chunks"] == 4 and st["wire_bytes"] == 8 * 4


def test_codec_narrowing_can_be_disabled(gpu_ctx, monkeypatch):
    """CBG_FIBER_* switches are read once per process; the default build takes the smallest form (checked above).
    Here: every chunk of a mixed product (one chunk varint-able, one with real values) picks its own form."""
    rng = np.random.default_rng(2)
    cols = [(np.arange(0, 500, 5), np.arange(1, 101, dtype=float)) for _ in range(8)]
    cols += [(np.arange(0, 500, 5), rng.standard_normal(100)) for _ in range(8)]
    st = _mat(gpu_ctx, 500, 16, cols).fiber_codec(2)
    _check(st, vals=(1 << 3) | (1 << 0))


def test_estimate_is_symbolic_and_exact(gpu_ctx):
    n, cp, ir, val = cb.generate_rmat_host(14, 16, seed=9)
    A = cb.SpDCCols.from_csc(gpu_ctx, n, n, cp, ir, val)
    m, z = cb.EstimateLocalNNZ(A, A)
    prof = gpu_ctx.last_profile()
    assert prof["numeric_ms"] == 0.0   # stopped after the symbolic pass and the scan
    C = cb.LocalSpGEMMHash(cb.PlusTimesSRing("f64"), A, A)
    assert (m, z) == (C.multiplies, C.getnnz())
    assert cb.EstimateLocalFLOP(cb.PlusTimesSRing("f64"), A, A) == m


def test_profile_heavy_counts(gpu_ctx):
    """cbg_profile.heavy_*: what the heavy kernels processed = the columns with nnz(C(:,j)) > 4096 (bench.py prices
    the dominant kernel's algorithmic bytes with these)."""
    n, cp, ir, val = cb.generate_rmat_host(16, 16, seed=3)
    A = cb.SpDCCols.from_csc(gpu_ctx, n, n, cp, ir, val)
    C = cb.LocalSpGEMMHash(cb.PlusTimesSRing("f64"), A, A)
    p = gpu_ctx.last_profile()
    ccp, _, _ = C.to_host()
    nz = np.diff(ccp)
    heavy = nz > K_HEAVY
    cnt = np.diff(cp)
    flop = np.array([cnt[ir[cp[j]:cp[j + 1]]].sum() for j in range(n)])
    assert heavy.any()
    assert p["heavy_multiplies"] == int(flop[heavy].sum())
    assert p["heavy_nnz_b"] == int(cnt[heavy].sum())
    assert p["heavy_nnz_c"] == int(nz[heavy].sum())


def test_codec_five_byte_varints_across_lanes_and_steps(gpu_ctx):
    """Varint integer values in [2^28, 2^32) take 5 bytes, the longest code: the decoder finds a code's start by looking
    back into the previous lane or the carried lane 63 of the previous 64-byte step.  Long columns (several thousand
    encoded bytes) with 5-byte codes at every offset modulo 64 -- so they straddle lane and step boundaries -- mixed
    with 1-byte codes, still choose the varint form and round trip bit for bit; rows with gaps of every code length."""
    rng = np.random.default_rng(17)
    n = (1 << 30) + 12345
    cols = []
    for c in range(6):
        m = 3000 + 17 * c
        gaps = rng.choice([1, 2, 200, 20000, 3_000_000], m, p=[0.6, 0.2, 0.1, 0.07, 0.03])
        rows = np.cumsum(gaps) - 1
        rows = rows[rows < n]
        v = rng.integers(0, 100, len(rows)).astype(np.float64)
        big = np.arange(c, len(rows), 37)                      # every offset mod 64 over the column
        v[big] = rng.integers(1 << 28, 1 << 32, len(big)).astype(np.float64)
        v[big[::5]] = float((1 << 32) - 1)                     # the largest u32
        cols.append((rows, v))
    st = _mat(gpu_ctx, n, len(cols), cols).fiber_codec(3)
    _check(st, vals=1 << 3)
    assert st["entries"] == sum(len(c[0]) for c in cols)


def test_codec_one_pass_equals_two_pass(gpu_ctx):
    """The one-pass encoder (k_code_encode: counts + codes into per-column slots, then packed) produces the same wire
    bytes and forms as the two-pass one (k_code_count, then k_var_encode re-reading the partial; CBG_FIBER_ONEPASS=0,
    read once per process, so it runs in a child process), and both round-trip bit for bit."""
    import json
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    script = (
        "import sys, json; sys.path.insert(0, %r)\n"
        "import numpy as np, combblas_amd as cb\n"
        "ctx = cb.Context(0)\n"
        "n, cp, ir, val = cb.generate_rmat_host(13, 16, seed=9)\n"
        "A = cb.SpDCCols.from_csc(ctx, n, n, cp, ir, val)\n"
        "C = cb.LocalSpGEMMHash(cb.PlusTimesSRing('f64'), A, A)\n"
        "print(json.dumps(C.fiber_codec(3)))\n") % os.path.dirname(here)
    outs = []
    for onepass in ("1", "0"):
        r = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=300,
                           env=dict(os.environ, CBG_FIBER_ONEPASS=onepass))
        assert r.returncode == 0, r.stderr[-2000:]
        outs.append(json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1]))
    for st in outs:
        _check(st, rows=1 << 2, vals=1 << 3)
    keys = ("wire_bytes", "row_bytes", "value_bytes", "value_header_bytes", "header_bytes", "entries")
    assert {k: outs[0][k] for k in keys} == {k: outs[1][k] for k in keys}
