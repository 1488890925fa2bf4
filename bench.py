#!/usr/bin/env python3
"""Benchmark: SpGEMM multiplies/s on R-MAT A*A (PlusTimes<double>) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scale S] [--no-cpu]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Without WORLD_SIZE in the environment, `--gpus N > 1` makes this process a launcher: it starts N rank processes of
this script (RANK / LOCAL_RANK / WORLD_SIZE set, one GPU each) before any GPU call, relays rank 0's JSON line and
exits non-zero if any rank fails.  Under torch.distributed.run, WORLD_SIZE must equal --gpus.

Workload (BASELINE.json configs): Graph500 Kronecker / R-MAT, edge factor 16, A*A over PlusTimes<double>,
inputs built on the GPU from the reference's own Graph500 edge stream (seed 0xDECAFBAD, the reference's
default SEED; the s20 matrix's hash equals refprobe `gen` output) and resident in HBM before the timed region.
  N = 1: configs[1], scale 20, the local hash SpGEMM (cbg_spgemm_local) on one GPU.
  N > 1: the distributed product on the mandated layout (combblas_amd/dist.py):
         2 -> 1x1x2, 4 -> 2x2 SUMMA, 8 -> 2x2x2 (configs[2] at scale 22), RCCL over xGMI.
         Default scale 20 + {2: 1, 4: 1, 8: 2}[N]: per-GPU work stays within ~1.5x of N = 1 ("weak").
One step = one complete product (column statistics, binning, symbolic, scan, allocation of C, numeric
with row-sorted output; for N > 1 also the stage broadcasts, partial merges and the fiber exchange).
K steps are timed between a barrier + device synchronisation on both sides, max over ranks; value =
all ranks' multiplies / that time.

Rank 0 prints ONE JSON line.  N = 1 adds `roofline` for the dominant phase (the heavy-column units:
k_num_heavy_known, plus k_num_heavy for the few units it does not take, bracketed by HIP events on the
library stream; algorithmic bytes per SURVEY §8d; `roofline.step` = the whole product) and `cpu_baseline`:
the reference's own LocalSpGEMMHash (oracle/_ref/refbench, built from /root/reference's sources) timed on a
bounded sample of the same product, its output checksum compared with the GPU product's (the oracle
restatement, also timed as `cpu_baseline_port`, checks the sample bit for bit).

    python bench.py --rank-share all --gpus-virtual 8 --scale 22
runs each rank's share of the N-GPU layout on this one GPU (local ms, fiber bytes, peak HBM; no transport).
"""
import argparse
import ctypes
import glob
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "SpGEMM multiplies/sec, R-MAT s22 A·A at 1/2/4/8 MI355X + achieved HBM GB/s"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
S_I, S_V, S_P = 4, 8, 8        # row-index, value, column-pointer bytes
K_HEAVY = 4096                 # nnz(C(:,j)) above which a column is split into units (spgemm_kernels.hpp)


def balg_bytes(mults, nnzc, nnzb, ncolb):
    """SURVEY §8(d) algorithmic bytes of one whole SpGEMM."""
    return (mults * (2 * S_I + S_V) + nnzc * (S_I + S_V) + nnzb * (2 * S_I + S_V + 4 * S_P)
            + 4 * (ncolb + 1) * S_P)


def heavy_bytes(flop_col, nnz_c_col, nnz_b_col, heavy):
    """SURVEY §8(d) numeric-phase algorithmic bytes of the heavy columns (what the heavy kernels process):
    gather A (row, val) per multiply, read B (row, val) + the A colptr pair per B nonzero, write C."""
    return (int(flop_col[heavy].sum()) * (S_I + S_V) + int(nnz_b_col[heavy].sum()) * (S_I + S_V + 2 * S_P)
            + int(nnz_c_col[heavy].sum()) * (S_I + S_V))


def round_tag(path):
    """Sort key of a profiles/ file by its evidence tag: r<round><letters>_..., letters in spreadsheet order
    (r03y < r03z < r03aa < r03aj), so the newest build's file sorts last."""
    import re
    m = re.match(r"r(\d+)([a-z]*)_", os.path.basename(path))
    if not m:
        return (-1, 0, "")
    return (int(m.group(1)), len(m.group(2)), m.group(2))


def load_traffic(scale, edgefactor):
    """HBM bytes per product of the heavy kernels from the newest committed rocprofv3 PMC summary for this
    workload (profiles/*_pmc_heavy.json, written by tools/pmc_heavy.py), or (None, None)."""
    best = None
    for f in sorted(glob.glob(os.path.join(HERE, "profiles", "*_pmc_heavy.json")), key=round_tag):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("scale") == scale and d.get("edgefactor") == edgefactor:
            best = (f, d)
    if best is None:
        return None, None
    return best[1]["bytes_per_launch"], os.path.relpath(best[0], HERE)


def load_step_traffic(scale, edgefactor):
    """HBM bytes of one whole product (every kernel) from the newest profiles/*_pmc_product.json for this
    workload (tools/pmc_heavy.py product), or (None, None)."""
    best = None
    for f in sorted(glob.glob(os.path.join(HERE, "profiles", "*_pmc_product.json")), key=round_tag):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("scale") == scale and d.get("edgefactor") == edgefactor:
            best = (f, d)
    if best is None:
        return None, None
    return best[1]["bytes_per_product"], os.path.relpath(best[0], HERE)


def col_flops(cp, ir):
    """estimateFLOP per column of A*A (mtSpGEMM.h:1117-1135)."""
    nnz_col = np.diff(cp)
    csum = np.concatenate([[0], np.cumsum(nnz_col[ir])])
    return csum[cp[1:]] - csum[cp[:-1]]


def sample_columns(n, flop_col, target_mults):
    """Every s-th column of B, s chosen so the sample holds about target_mults multiplies."""
    tot = int(flop_col.sum())
    stride = max(1, int(np.ceil(tot / max(target_mults, 1))))
    return np.arange(0, n, stride), stride


def host_cores(n_gpus_visible=1):
    """Host threads for the CPU baselines: the cores this process may run on (affinity), capped by a cgroup CPU quota
    and by the pool's share of 16 cores per visible GPU (os.cpu_count() shows the whole machine there).  Returns
    (threads, record of every figure)."""
    import math
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    threads = aff
    if quota:
        threads = min(threads, max(1, math.floor(quota)))
    share = 16 * max(1, n_gpus_visible)
    threads = max(1, min(threads, share))
    return threads, {"os_cpu_count": os.cpu_count(), "affinity_cpus": aff, "cgroup_quota_cpus": quota,
                     "pool_share_cpus": share, "OMP_NUM_THREADS_env": os.environ.get("OMP_NUM_THREADS")}


def cpu_baseline(cp, ir, val, n, flop_col, target_mults):
    """Oracle (CPU restatement, oracle/oracle.c) on a bounded sample: every s-th column of B.
    Returns (baseline JSON, the oracle's product of the sampled columns)."""
    sys.path.insert(0, os.path.join(HERE, "tests"))
    from helpers import Csc, oracle_spgemm  # test infrastructure: checker/baseline only
    cols, stride = sample_columns(n, flop_col, target_mults)
    bcp = np.concatenate([[0], np.cumsum(np.diff(cp)[cols])]).astype(np.int64)
    idx = np.concatenate([np.arange(cp[c], cp[c + 1]) for c in cols]) if len(cols) else np.zeros(0, np.int64)
    A = Csc(n, n, cp, ir, val)
    B = Csc(n, len(cols), bcp, ir[idx], val[idx])
    threads, _ = host_cores(_visible_gpus())
    os.environ["OMP_NUM_THREADS"] = str(threads)   # the oracle's OpenMP pool starts on first use, in this process
    t0 = time.perf_counter()
    C, mults, rc = oracle_spgemm(A, B, "plus_times", "f64")
    dt = time.perf_counter() - t0
    assert rc == 0
    return ({"value": mults / dt, "unit": "multiplies/s", "cores": threads, "kind": "port",
             "sample": f"oracle/oracle.c (CPU restatement of LocalSpGEMMHash, OpenMP, {threads} threads) on "
                       f"every {stride}-th column of B ({len(cols)} columns, {mults} multiplies, {dt:.2f} s)"},
            (cols, C))


def _visible_gpus():
    try:
        import torch
        return max(1, torch.cuda.device_count())
    except Exception:
        return 1


def verify_sample(Cdev, cols, R):
    """Bit-exact check of the benchmarked product on the sampled columns against the oracle's product
    of the same columns (R-MAT values are multiplicities, so PlusTimes<double> sums are exact).
    Also returns the sampled columns' entry checksum (compared with the reference's own product)."""
    S = Cdev.select_columns(cols)
    scp, sir, sval = S.to_host()
    S.free()
    ok = bool(np.array_equal(scp, R.cp) and np.array_equal(sir, R.ir) and np.array_equal(sval, R.val))
    return ({"columns": int(len(cols)), "nnz": int(R.cp[-1]), "bit_exact": ok,
             "against": "oracle/oracle.c product of the cpu_baseline sample columns"},
            entry_checksum(scp, sir, sval))


REFBENCH = os.path.join(HERE, "oracle", "_ref", "refbench")


def _s64(u):
    return u - (1 << 64) if u >= 1 << 63 else u


_MIX = [_s64(0x9E3779B97F4A7C15), _s64(0xBF58476D1CE4E5B9), _s64(0x94D049BB133111EB)]


def _lsr(x, k):
    """Logical right shift of an int64 tensor (two's complement bits)."""
    return (x >> k) & ((1 << (64 - k)) - 1)


def _mix64_t(x):
    """splitmix64 finaliser on an int64 torch tensor (wrapping arithmetic = the uint64 bits of _mix64)."""
    x = x + _MIX[0]
    x = (x ^ _lsr(x, 30)) * _MIX[1]
    x = (x ^ _lsr(x, 27)) * _MIX[2]
    return x ^ _lsr(x, 31)


def entry_checksum_t(cols, rows, val):
    """entry_checksum's sum over the entries (global col ids, rows, f64 values as torch tensors on any device), as an
    int64 whose bits are the uint64 sum mod 2^64 -- summable over ranks."""
    import torch
    if rows.numel() == 0:
        return 0
    h = _mix64_t((rows.to(torch.int64) << 32) ^ cols.to(torch.int64)) ^ _mix64_t(val.contiguous().view(torch.int64))
    return int(h.sum().item())


def _mix64(x):
    """splitmix64 finaliser on uint64 arrays (wrapping), as oracle/ref/refbench.cpp's mix64."""
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))


def entry_checksum(cp, ir, val, chunk=1 << 24):
    """Order-independent checksum of a CSC's entries: sum of mix(row << 32 ^ col) ^ mix(value bits) mod 2^64
    (oracle/ref/refbench.cpp computes the same over the reference's output tuples)."""
    cols = np.repeat(np.arange(len(cp) - 1, dtype=np.uint64), np.diff(cp))
    bits = np.ascontiguousarray(val, np.float64).view(np.uint64)
    s = np.uint64(0)
    with np.errstate(over="ignore"):
        for a in range(0, len(ir), chunk):
            r = ir[a:a + chunk].astype(np.uint64)
            h = _mix64((r << np.uint64(32)) ^ cols[a:a + chunk]) ^ _mix64(bits[a:a + chunk])
            s = s + np.sum(h, dtype=np.uint64)
    return f"{int(s):016x}"


def reference_baseline(n, cp, ir, val, stride, threads, synch_factor=3):
    """The reference's own CPU SpGEMM (oracle/_ref/refbench, compiled from /root/reference's sources by
    oracle/ref/Makefile) timed on the same sample: LocalSpGEMMHash on every `stride`-th column of B, and the
    1-rank Mult_AnXBn_Synch (local hash + MultiwayMerge + DCSC build) on every (synch_factor*stride)-th column.
    Returns the parsed JSON lines, or None when the binary is absent."""
    import subprocess
    import tempfile
    if not os.path.exists(REFBENCH):
        return None
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "A.bin")
        with open(path, "wb") as f:   # CBM1 (oracle/ref/refprobe.cpp): f64 values, int64 indices
            f.write(b"CBM1")
            np.array([0], np.int32).tofile(f)
            np.array([n, n, len(ir)], np.int64).tofile(f)
            np.asarray(cp, np.int64).tofile(f)
            np.asarray(ir, np.int64).tofile(f)
            np.asarray(val, np.float64).tofile(f)
        env = dict(os.environ, OMP_NUM_THREADS=str(threads))
        r = subprocess.run([REFBENCH, path, str(stride), str(stride * synch_factor)], capture_output=True, text=True,
                           env=env, timeout=600)
    if r.returncode != 0:
        print(f"bench: refbench failed ({r.returncode}): {r.stderr[-2000:]}", file=sys.stderr)
        return None
    return {d["call"]: d for d in (json.loads(x) for x in r.stdout.splitlines() if x.startswith("{"))}


def input_record(args, cp, ir, val, build_s):
    """How the input was made, and whether it is the reference's own matrix: the canonical SHA-256 of the
    device-built matrix against the hash of refprobe `gen` output for the same scale/seed
    (tests/golden/kron.json, made by tests/golden/make_golden_kron.py from the reference build)."""
    sys.path.insert(0, os.path.join(HERE, "tests", "golden"))
    from cbm import canonical_sha256
    rec = {"generator": "cbg_generate_rmat on the GPU: the reference's Graph500 edge stream (RefGen21, packed) + "
                        "duplicate-summing build (SpParMat(DistEdgeList))", "seed": args.seed,
           "device_build_s": round(build_s, 4), "nnz": int(len(ir))}
    try:
        ref = [c for c in json.load(open(os.path.join(HERE, "tests", "golden", "kron.json")))["cases"]
               if (c["scale"], c["edgefactor"], c["seed"]) == (args.scale, args.edgefactor, args.seed)]
    except (OSError, ValueError):
        ref = []
    if ref:
        rec["sha256_equals_reference_generator"] = canonical_sha256(cp, ir, val) == ref[0]["sha256"]
    return rec


def workload(scale, edgefactor, parallelism):
    return {"workload": f"R-MAT (Graph500 Kronecker a,b,c,d=.57,.19,.19,.05, scrambled ids, duplicates summed) "
                        f"scale-{scale} edge factor {edgefactor} A*A PlusTimes<double>",
            "scale": scale, "edgefactor": edgefactor, "parallelism": parallelism}


# ------------------------------------------------------------------------------------------ N = 1
def bench_local(args):
    import combblas_amd as cb
    from combblas_amd import _abi

    ctx = cb.Context(0)
    t0 = time.perf_counter()
    A = ctx.generate_rmat(args.scale, args.edgefactor, seed=args.seed)   # built in HBM (kron.hip)
    ctx.synchronize()
    build_s = time.perf_counter() - t0
    n = A.getncol()
    cp, ir, val = A.to_host()            # host copy: column statistics, CPU baseline, input hash
    flop_col = col_flops(cp, ir)
    va = A._view()
    lib = ctx._lib
    keep = {}

    def step(keep_colptr=False, keep_result=False):
        res = _abi.CscResult()
        m = ctypes.c_int64()
        _abi.check(lib.cbg_spgemm_local(ctx._ptr, ctypes.byref(va), ctypes.byref(va), _abi.SR_PLUS_TIMES,
                                        _abi.F64, _abi.SORTED_COLS, ctypes.byref(res), ctypes.byref(m)),
                   "cbg_spgemm_local")
        prof = ctx.last_profile()
        if keep_colptr:   # structure of C, outside the timed region: which columns were heavy
            ccp = np.zeros(int(res.ncol) + 1, np.int64)
            _abi.check(lib.cbg_result_to_host(ctx._ptr, ctypes.byref(res), ccp.ctypes.data, None, None))
            keep["cp"] = ccp
        nnzc = int(res.nnz)
        if keep_result:   # the last timed product is kept for the parity check (no extra work timed)
            keep["C"] = cb.SpDCCols._from_result(ctx, res)
        else:
            lib.cbg_result_free(ctx._ptr, ctypes.byref(res))
        return int(m.value), nnzc, prof

    for w in range(max(args.warmup, 1)):
        step(keep_colptr=(w == 0))
    ctx.synchronize()
    t0 = time.perf_counter()
    mults = nnzc = 0
    profs = []
    for s in range(args.steps):
        m, z, prof = step(keep_result=(s == args.steps - 1))
        mults += m
        nnzc += z
        profs.append(prof)
    ctx.synchronize()
    elapsed = time.perf_counter() - t0

    nnz_c_col = np.diff(keep["cp"])
    heavy = nnz_c_col > K_HEAVY
    mult_step, nnzc_step = mults / args.steps, nnzc / args.steps
    nnzb = int(cp[-1])
    hb = heavy_bytes(flop_col, nnz_c_col, np.diff(cp), heavy)
    heavy_ms = float(np.mean([p["heavy_ms"] for p in profs]))
    achieved = hb / (heavy_ms / 1e3) / 1e9
    traffic, tsrc = load_traffic(args.scale, args.edgefactor)
    step_traffic, ssrc = load_step_traffic(args.scale, args.edgefactor)
    cfg = workload(args.scale, args.edgefactor, "single GPU, local hash SpGEMM (BASELINE configs[1])")
    cfg.update({"nnz_A": nnzb, "multiplies": int(mult_step), "nnz_C": int(nnzc_step)})
    out = {
        "metric": METRIC, "value": mults / elapsed, "unit": "multiplies/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": 1000.0 * elapsed / args.steps, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic", "config": cfg,
        "effective_GBps": balg_bytes(mult_step, nnzc_step, nnzb, n) / (elapsed / args.steps) / 1e9,
        "phases_ms": {k: round(float(np.mean([p[k] for p in profs])), 3)
                      for k in ("flops_ms", "bin_ms", "symbolic_ms", "scan_ms", "numeric_ms", "heavy_ms",
                                "total_ms")},
        "heavy_items": {"items": int(profs[-1]["bins"][13]), "rows_known_units": int(profs[-1]["known_items"])},
        "roofline": {"bound": "hbm", "kernel": "k_num_heavy_known + k_num_heavy (heavy-column units)", "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_source": tsrc, "algorithmic_bytes_per_launch": hb, "avg_launch_ms": heavy_ms,
                     "heavy_columns": int(heavy.sum()), "heavy_multiplies": int(flop_col[heavy].sum()),
                     "heavy_nnz_C": int(nnz_c_col[heavy].sum()),
                     # the whole product (every kernel): SURVEY 8(d) algorithmic bytes vs PMC FETCH+WRITE
                     "step": {"algorithmic_bytes": balg_bytes(mult_step, nnzc_step, nnzb, n),
                              "achieved_GBps": balg_bytes(mult_step, nnzc_step, nnzb, n) / (elapsed / args.steps) / 1e9,
                              "traffic": step_traffic, "traffic_source": ssrc}},
    }
    out["input"] = input_record(args, cp, ir, val, build_s)
    if not args.no_cpu:
        port, (cols, R) = cpu_baseline(cp, ir, val, n, flop_col, args.cpu_mults)
        out["verified"], gpu_sum = verify_sample(keep["C"], cols, R)
        keep.pop("C").free()
        stride = int(cols[1] - cols[0]) if len(cols) > 1 else 1
        ref = reference_baseline(n, cp, ir, val, stride, port["cores"])
        if ref and "LocalSpGEMMHash" in ref:
            h = ref["LocalSpGEMMHash"]
            out["cpu_baseline"] = {
                "value": h["multiplies"] / h["seconds"], "unit": "multiplies/s", "cores": h["omp_threads"],
                "mpi_ranks": h["mpi_ranks"], "omp_threads": h["omp_threads"], "kind": "reference",
                "host": host_cores(_visible_gpus())[1],
                "sample": f"the reference's LocalSpGEMMHash<PlusTimesSRing<double,double>> (mtSpGEMM.h:465-661, "
                          f"oracle/_ref/refbench built from /root/reference sources, -O3 -fopenmp) at 1 MPI rank x "
                          f"{h['omp_threads']} OpenMP threads on every {stride}-th column of B ({h['columns']} columns, "
                          f"{h['multiplies']} multiplies, {h['seconds']:.2f} s)"}
            out["verified"]["reference_checksum_equal"] = h["checksum"] == gpu_sum and h["nnzC"] == out["verified"]["nnz"]
            s = ref.get("Mult_AnXBn_Synch")
            if s:
                out["cpu_baseline"]["synch"] = {
                    "value": s["multiplies"] / s["seconds"], "unit": "multiplies/s",
                    "sample": f"Mult_AnXBn_Synch (ParFriends.h:1004-1108: local hash + MultiwayMerge + DCSC build), "
                              f"1 rank x {s['omp_threads']} threads, every {s['stride']}-th column "
                              f"({s['multiplies']} multiplies, {s['seconds']:.2f} s)"}
            out["cpu_baseline_port"] = port
        else:
            out["cpu_baseline"] = port
    else:
        keep.pop("C").free()
    print(json.dumps(out), flush=True)
    if not args.no_cpu and not out["verified"]["bit_exact"]:
        sys.exit("bench: the benchmarked product differs from the oracle on the sampled columns")


# ------------------------------------------------------------------------------------------ N > 1
def select_block_cols(b, cols):
    """Columns `cols` (sorted local ids, int64 tensor) of a Block, as a Block on the same device."""
    import torch
    from combblas_amd import dist as cbd
    cols = cols.to(device=b.cp.device, dtype=torch.int64)
    s, e = b.cp[cols], b.cp[cols + 1]
    ln = e - s
    cp = torch.zeros(cols.numel() + 1, dtype=torch.int64, device=b.cp.device)
    torch.cumsum(ln, 0, out=cp[1:])
    tot = int(cp[-1].item())
    idx = torch.repeat_interleave(s - cp[:-1], ln, output_size=tot) + torch.arange(tot, device=b.cp.device)
    return cbd.Block(b.nrow, int(cols.numel()), cp, b.ir[idx], b.val[idx])


def piece_reference(be, args, n, r0, r1, c0, c1):
    """What a rank's output piece C(r0:r1, c0:c1) must be made of, built on the rank's own GPU independently of the
    grid: A(r0:r1, :) and A(:, c0:c1) from the reference's generator, and the symbolic pass (estimateFLOP + exact
    nnz) of their product."""
    Arow = be.rmat_block(args.scale, args.edgefactor, args.seed, r0, r1, 0, n)
    Acol = be.rmat_block(args.scale, args.edgefactor, args.seed, 0, n, c0, c1)
    mults, nnz = be.estimate(Arow, Acol)
    return Arow, Acol, mults, nnz


def piece_checksum(blk, r0, c0, chunk=1 << 27):
    """entry_checksum_t over a whole output piece (global row and column ids), in column chunks of about `chunk`
    entries: summed over the ranks it is the checksum of the whole distributed product, the same for every layout of
    one product (SURVEY 8(d)'s cross-layout identity; R-MAT values are multiplicities, so every layout's sums are
    bit-identical)."""
    import torch
    cp = blk.cp
    ncol = blk.ncol
    total = 0
    a = 0
    cph = cp.cpu().numpy()
    while a < ncol:
        b = int(np.searchsorted(cph, cph[a] + chunk, side="right")) - 1
        b = min(ncol, max(b, a + 1))
        lo, hi = int(cph[a]), int(cph[b])
        if hi > lo:
            cols = torch.repeat_interleave(torch.arange(a, b, device=cp.device, dtype=torch.int64) + c0,
                                           torch.diff(cp[a:b + 1]), output_size=hi - lo)
            total = (total + entry_checksum_t(cols, blk.ir[lo:hi].to(torch.int64) + r0, blk.val[lo:hi])) & ((1 << 64) - 1)
        a = b
    return total - (1 << 64) if total >= 1 << 63 else total


def oracle_piece_sample(blk, Arow, Acol, ncols, seed):
    """The CHECKER's leg of the distributed checks (test infrastructure, never timed): a seeded sample of `ncols`
    columns of a rank's output piece against oracle/oracle.c's product A(rows_i, :) * A(:, J_sample) on the host (the
    reference-pinned restatement of LocalSpGEMMHash, mtSpGEMM.h:465-661), bit for bit (R-MAT multiplicities)."""
    import torch
    sys.path.insert(0, os.path.join(HERE, "tests"))
    from helpers import Csc, oracle_spgemm  # test infrastructure: checker only
    k = min(blk.ncol, int(ncols))
    g = torch.Generator().manual_seed(int(seed) ^ 0x5EED)
    sel = torch.randperm(blk.ncol, generator=g)[:k].sort().values
    B = select_block_cols(Acol, sel)
    S = select_block_cols(blk, sel)
    A = Csc(Arow.nrow, Arow.ncol, Arow.cp.cpu().numpy(), Arow.ir.cpu().numpy(), Arow.val.cpu().numpy())
    Bh = Csc(B.nrow, B.ncol, B.cp.cpu().numpy(), B.ir.cpu().numpy(), B.val.cpu().numpy())
    R, mults, rc = oracle_spgemm(A, Bh, "plus_times", "f64")
    ok = (rc == 0 and np.array_equal(S.cp.cpu().numpy(), R.cp) and np.array_equal(S.ir.cpu().numpy(), R.ir)
          and np.array_equal(S.val.cpu().numpy().view(np.int64), np.asarray(R.val, np.float64).view(np.int64)))
    return {"oracle_sample_columns": k, "oracle_sample_nnz": int(R.cp[-1]), "oracle_sample_multiplies": int(mults),
            "oracle_sample": bool(ok)}


def verify_piece(be, SR, blk, Arow, Acol, r0, c0, nsample, seed, ref_stride=0, oracle_cols=0):
    """Check one rank's output piece: a seeded random sample of its columns bit for bit against a one-GPU product
    A(r0:r1, :) * A(:, J_sample) (R-MAT values are multiplicities, so PlusTimes<double> sums are exact), and the
    reference-sample checksum: entry_checksum over the piece's columns j = 0 mod ref_stride (global row ids, column
    id j // ref_stride), summable over ranks into the checksum of oracle/_ref/refbench's product of those columns."""
    import torch
    ncols = blk.ncol
    k = min(ncols, int(nsample))
    g = torch.Generator().manual_seed(int(seed))
    sel = torch.randperm(ncols, generator=g)[:k].sort().values
    P = be.multiply(Arow, select_block_cols(Acol, sel), SR)
    S = select_block_cols(blk, sel)
    exact = bool(P.nnz == S.nnz and torch.equal(P.cp, S.cp) and torch.equal(P.ir, S.ir)
                 and torch.equal(P.val.view(torch.int64), S.val.view(torch.int64)))
    rec = {"sampled_columns": k, "sample_nnz": P.nnz, "bit_exact": exact}
    del P, S
    if oracle_cols:
        rec.update(oracle_piece_sample(blk, Arow, Acol, oracle_cols, seed))
        rec["bit_exact"] = rec["bit_exact"] and rec["oracle_sample"]
    if ref_stride:
        first = (-c0) % ref_stride
        jl = torch.arange(first, ncols, ref_stride, dtype=torch.int64)
        R = select_block_cols(blk, jl)
        cols = torch.repeat_interleave((jl.to(R.cp.device) + c0) // ref_stride, torch.diff(R.cp), output_size=R.nnz)
        rec["ref_sample_nnz"] = R.nnz
        rec["ref_sample_checksum"] = entry_checksum_t(cols, R.ir.to(torch.int64) + r0, R.val)
    return rec


def local_roofline(st, ms_key="local_ms"):
    """SURVEY 8(d) algorithmic bytes of a rank's local products (grid stats summed over its products): the heavy
    kernels' share (the dominant kernel) and the whole local products."""
    hb = (st.get("heavy_multiplies", 0) * (S_I + S_V) + st.get("heavy_nnz_b", 0) * (S_I + S_V + 2 * S_P)
          + st.get("heavy_nnz_c", 0) * (S_I + S_V))
    lb = balg_bytes(st.get("multiplies", 0), st.get("local_nnz_out", 0), st.get("local_nnz_b", 0),
                    st.get("local_ncol_b", 0))
    return hb, lb


def bench_dist(args, world, rank, local_rank):
    import torch
    import torch.distributed as dist
    import combblas_amd as cb
    from combblas_amd import dist as cbd

    # production: RCCL, one GPU per rank.  Rehearsals with ranks sharing the visible GPUs (a one-GPU box):
    #   CBG_DIST_BACKEND=rccl-net  the same libcbgpu RCCL grid, every rank its own RCCL "node"
    #                              (NCCL_HOSTID) so RCCL's socket transport carries the bytes;
    #   CBG_DIST_BACKEND=gloo      the host-staged gloo transport.
    backend = os.environ.get("CBG_DIST_BACKEND", "nccl")
    if backend not in ("nccl", "rccl-net", "gloo"):
        sys.exit(f"bench: CBG_DIST_BACKEND={backend!r}: expected nccl, rccl-net or gloo")
    dev = local_rank % torch.cuda.device_count()
    torch.cuda.set_device(dev)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    else:
        if backend == "rccl-net":
            os.environ.update({"NCCL_HOSTID": f"cbg-bench-rank-{rank}", "NCCL_SOCKET_IFNAME": "lo",
                               "NCCL_IB_DISABLE": "1", "CBG_GRID_TRANSPORT": "rccl"})
        dist.init_process_group("gloo")
    ctx = cb.Context(dev)
    be = cbd.GpuBackend(ctx)
    n = 1 << args.scale
    if args.layout == "1d":
        return bench_1d(args, world, rank, ctx, be, n, backend)
    L, q, _ = cbd.grid_for(world)
    grid = cbd.CommGrid3D(L, q, q)
    t0 = time.perf_counter()
    # every rank builds only its own pieces, on its GPU (SpParMat3D.from_rmat -> cbg_rmat_block)
    A = cbd.SpParMat3D.from_rmat(grid, args.scale, args.edgefactor, args.seed, True, be)
    B = cbd.SpParMat3D.from_rmat(grid, args.scale, args.edgefactor, args.seed, False, be)
    torch.cuda.synchronize()
    build_s = time.perf_counter() - t0
    nnzb = A.getnnz()
    SR = cb.PlusTimesSRing("f64")

    phases = {}
    keep = {}

    def step(keep_result=False):
        st = {}
        C = cbd.Mult_AnXBn_SUMMA3D(SR, A, B, st)
        nz = C.block.nnz
        if keep_result:   # the last timed product is kept for the checks below (no extra work timed)
            keep["C"] = C
        del C
        for k, v in st.items():
            if isinstance(v, (int, float)):
                phases[k] = phases.get(k, 0) + v
        keep["fiber_mode"] = st.get("fiber_mode", "none")   # the grid's two-layer fiber step (gather / reduce)
        return st.get("multiplies", 0), nz

    step()   # first product also sets up libcbgpu's grid (its RCCL communicators); a failure ends the run
    ginfo = be.native_grid(grid).info()
    if backend != "gloo" and (ginfo["kind"] != "rccl" or ginfo["ranks"] != {"world": world, "row": q, "col": q,
                                                                          "fiber": L}):
        sys.exit(f"bench: libcbgpu grid is not the RCCL grid of a {L}x{q}x{q} layout: {ginfo}")
    for _ in range(max(args.warmup - 1, 0)):
        step()
    phases.clear()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    mults = nnzc = 0
    nzs = []
    for s_ in range(args.steps):
        m, z = step(keep_result=(s_ == args.steps - 1))
        mults += m
        nnzc += z
        nzs.append(z)
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    cd = be.comm_device
    t = torch.tensor([elapsed], dtype=torch.float64, device=cd)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed_local = elapsed
    s = torch.tensor([mults, nnzc], dtype=torch.float64, device=cd)
    dist.all_reduce(s)
    elapsed, mults, nnzc = float(t.item()), float(s[0].item()), float(s[1].item())

    # ---- checks, outside the timed region: every rank's piece against its independent reference
    C = keep.pop("C")
    (r0, r1), (c0, c1) = C.local_range()
    Arow, Acol, est_m, est_z = piece_reference(be, args, n, r0, r1, c0, c1)
    tot = torch.tensor([est_m, est_z], dtype=torch.int64, device=cd)
    dist.all_reduce(tot)
    flops_global, nnz_global = int(tot[0].item()), int(tot[1].item())
    ref_stride = max(1, int(np.ceil(flops_global / max(args.cpu_mults, 1)))) if not args.no_cpu else 0
    nsample = max(int(np.ceil(1e4 / world)), C.block.ncol // 64)
    v = verify_piece(be, SR, C.block, Arow, Acol, r0, c0, nsample, args.seed + 7919 * rank, ref_stride,
                     oracle_cols=0 if args.no_cpu else 256)
    v.update({"rank": rank, "rows": [r0, r1], "cols": [c0, c1], "piece_nnz": C.block.nnz,
              "piece_nnz_equals_estimate": C.block.nnz == est_z, "steps_same_nnz": len(set(nzs)) == 1})
    del Arow, Acol
    # per-rank roofline of the local products over the timed steps (grid stats), gathered with the checks
    hb, lb = local_roofline(phases)
    rrec = {"heavy_bytes": hb / args.steps, "heavy_ms": phases.get("heavy_ms", 0.0) / args.steps,
            "local_bytes": lb / args.steps, "local_ms": phases.get("local_ms", 0.0) / args.steps,
            "step_ms": 1e3 * elapsed_local / args.steps}
    recs = [None] * world
    dist.all_gather_object(recs, {"verify": v, "roofline": rrec, "phases": {k: w / args.steps for k, w in phases.items()}})
    csum = torch.tensor([v.get("ref_sample_checksum", 0), v.get("ref_sample_nnz", 0),
                         piece_checksum(C.block, r0, c0)], dtype=torch.int64, device=cd)
    dist.all_reduce(csum)   # int64 sums wrap: the uint64 checksum mod 2^64
    ok_all = all(r["verify"]["bit_exact"] and r["verify"]["piece_nnz_equals_estimate"] and r["verify"]["steps_same_nnz"]
                 for r in recs)
    ok_all = ok_all and int(mults / args.steps) == flops_global and int(nnzc / args.steps) == nnz_global
    fiber_mode = keep.get("fiber_mode", "none")
    keep.clear()
    del C
    torch.cuda.empty_cache()

    if rank == 0:
        cfg = workload(args.scale, args.edgefactor,
                       f"{L}x{q}x{q} ({'3D split SUMMA' if L > 1 else '2D SUMMA'}), "
                       f"libcbgpu grid over {ginfo['kind']}")
        cfg.update({"nnz_A": nnzb, "multiplies": int(mults / args.steps), "nnz_C": int(nnzc / args.steps)})
        slow = max(range(world), key=lambda r: recs[r]["roofline"]["local_ms"])
        rs = recs[slow]["roofline"]
        ach = rs["heavy_bytes"] / (rs["heavy_ms"] / 1e3) / 1e9 if rs["heavy_ms"] > 0 else 0.0
        ngpu = torch.cuda.device_count()
        rehearsal = backend != "nccl" or world > ngpu
        kern = ("k_num_heavy_known + k_num_heavy on the slowest rank (its local products per step; HIP events on the "
                "library stream)")
        if rehearsal:
            kern = (f"REHEARSAL, not a hardware roofline: {world} ranks share {ngpu} GPU(s) over {backend}; " + kern)
        out = {"metric": METRIC, "value": mults / elapsed, "unit": "multiplies/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1000.0 * elapsed / args.steps,
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
               "data": "synthetic", "config": cfg,
               "effective_GBps": balg_bytes(mults / args.steps, nnzc / args.steps, nnzb, n)
               / (elapsed / args.steps) / 1e9,
               "roofline": {"bound": "hbm (rehearsal)" if rehearsal else "hbm", "kernel": kern, "rehearsal": rehearsal,
                            "rank": slow, "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": ach / HBM_PEAK_GBS, "traffic": None,
                            "algorithmic_bytes_per_step": rs["heavy_bytes"], "avg_ms_per_step": rs["heavy_ms"],
                            "step": {"local_algorithmic_bytes": rs["local_bytes"], "local_ms": rs["local_ms"],
                                     "local_GBps": rs["local_bytes"] / (rs["local_ms"] / 1e3) / 1e9
                                     if rs["local_ms"] > 0 else 0.0, "rank_step_ms": rs["step_ms"]},
                            "per_rank": [{k: round(x, 3) if isinstance(x, float) else x for k, x in r["roofline"].items()}
                                         for r in recs]},
               "verified": {"bit_exact": all(r["verify"]["bit_exact"] for r in recs),
                            "sampled_columns": sum(r["verify"]["sampled_columns"] for r in recs),
                            "sampled_nnz": sum(r["verify"]["sample_nnz"] for r in recs),
                            "against": "per rank: a seeded sample of its output columns vs a one-GPU product "
                                       "A(rows_i, :) * A(:, J_sample) built independently of the grid (cbg_rmat_block), "
                                       "and 256 of them vs oracle/oracle.c's product on the host (oracle_sample)",
                            "oracle_sample": all(r["verify"].get("oracle_sample", False) for r in recs),
                            "multiplies_equal_estimateFLOP": int(mults / args.steps) == flops_global,
                            "nnz_equal_symbolic": int(nnzc / args.steps) == nnz_global,
                            "estimateFLOP": flops_global, "nnz_symbolic": nnz_global, "ok": ok_all,
                            "per_rank": [r["verify"] for r in recs]},
               "rank0_phases_per_step": {k: round(w, 3) for k, w in recs[0]["phases"].items()},
               # the whole product's entry checksum (every rank's piece): equal across the layouts of one scale
               "full_output_checksum": f"{int(csum[2].item()) & ((1 << 64) - 1):016x}",
               "grid_transport": ginfo["kind"],
               "fiber_mode": fiber_mode,
               # members of every communicator as RCCL itself counts them (ncclCommCount)
               "rccl_ranks": ginfo["ranks"] if ginfo["kind"] == "rccl" else None,
               "input": {"generator": "SpParMat3D.from_rmat: each rank builds its own A and B pieces on its GPU "
                                      "(cbg_rmat_block, the reference's Graph500 edge stream)", "seed": args.seed,
                         "rank0_device_build_s": round(build_s, 4), "nnz": nnzb}}
        if not args.no_cpu:
            # the reference's own CPU SpGEMM on every ref_stride-th column of the global product (rank 0's host
            # cores), its output checksum against the sum of the ranks' checksums of the same columns
            Ag = ctx.generate_rmat(args.scale, args.edgefactor, seed=args.seed)
            cp, ir, val = Ag.to_host()
            Ag.free()
            threads, host = host_cores(_visible_gpus())
            ref = reference_baseline(n, cp, ir, val, ref_stride, threads)
            del cp, ir, val
            if ref and "LocalSpGEMMHash" in ref:
                h = ref["LocalSpGEMMHash"]
                out["cpu_baseline"] = {
                    "value": h["multiplies"] / h["seconds"], "unit": "multiplies/s", "cores": h["omp_threads"],
                    "mpi_ranks": h["mpi_ranks"], "omp_threads": h["omp_threads"], "kind": "reference", "host": host,
                    "sample": f"the reference's LocalSpGEMMHash<PlusTimesSRing<double,double>> (mtSpGEMM.h:465-661, "
                              f"oracle/_ref/refbench) at 1 MPI rank x {h['omp_threads']} OpenMP threads on rank 0's "
                              f"host, every {ref_stride}-th column of B ({h['columns']} columns, {h['multiplies']} "
                              f"multiplies, {h['seconds']:.2f} s)"}
                got = f"{int(csum[0].item()) & ((1 << 64) - 1):016x}"
                out["verified"]["reference_checksum_equal"] = (h["checksum"] == got
                                                               and h["nnzC"] == int(csum[1].item()))
                out["verified"]["reference_sample"] = {"stride": ref_stride, "nnz": h["nnzC"],
                                                       "checksum_reference": h["checksum"], "checksum_grid": got}
                ok_all = ok_all and out["verified"]["reference_checksum_equal"]
                out["verified"]["ok"] = ok_all
        print(json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    if not ok_all:
        sys.exit("bench: the distributed product failed its checks (verified.per_rank)")


def bench_1d(args, world, rank, ctx, be, n, backend):
    """SURVEY §8(e)'s stated comparison (not the mandated layouts): a 1D column split.  Rank r builds its column
    block A(:, J_r) on its GPU; every step all-gathers the blocks (A replicated: one RCCL all-gather of counts,
    rows and values) and multiplies A * A(:, J_r) locally -- C(:, J_r) complete, no merge, no fiber exchange."""
    import torch
    import torch.distributed as dist
    import combblas_amd as cb
    from combblas_amd import dist as cbd
    c0, c1 = cbd.block_range(n, world, rank)
    t0 = time.perf_counter()
    mine = be.rmat_block(args.scale, args.edgefactor, args.seed, 0, n, c0, c1)   # rows 0..n-1, columns J_r
    torch.cuda.synchronize()
    build_s = time.perf_counter() - t0
    cd = be.comm_device
    widths = [cbd.block_range(n, world, r)[1] - cbd.block_range(n, world, r)[0] for r in range(world)]
    nz = torch.tensor([mine.nnz], dtype=torch.int64, device=cd)
    nzs = [torch.zeros(1, dtype=torch.int64, device=cd) for _ in range(world)]
    dist.all_gather(nzs, nz)
    nzs = [int(x.item()) for x in nzs]
    mx = max(nzs)
    SR = cb.PlusTimesSRing("f64")
    phases = {}

    def gather_a():
        cnt = torch.diff(mine.cp).to(cd)
        ir = torch.zeros(mx, dtype=torch.int32, device=cd)
        val = torch.zeros(mx, dtype=torch.float64, device=cd)
        ir[:mine.nnz] = mine.ir.to(cd)
        val[:mine.nnz] = mine.val.to(cd)
        wmax = max(widths)
        cntp = torch.zeros(wmax, dtype=torch.int64, device=cd)
        cntp[:cnt.numel()] = cnt
        outs = []
        for t, proto in ((cntp, wmax), (ir, mx), (val, mx)):
            g = torch.empty(world * proto, dtype=t.dtype, device=cd)
            dist.all_gather_into_tensor(g, t)
            outs.append(g)
        cnts = torch.cat([outs[0][r * wmax:r * wmax + widths[r]] for r in range(world)])
        irs = torch.cat([outs[1][r * mx:r * mx + nzs[r]] for r in range(world)])
        vals = torch.cat([outs[2][r * mx:r * mx + nzs[r]] for r in range(world)])
        cp = torch.zeros(n + 1, dtype=torch.int64, device=cd)
        torch.cumsum(cnts, 0, out=cp[1:])
        return cbd.Block(n, n, cp.to(be.device), irs.to(be.device), vals.to(be.device))

    def step():
        ta = time.perf_counter()
        Afull = gather_a()
        torch.cuda.synchronize()
        tb = time.perf_counter()
        st = {}
        C = be.multiply(Afull, mine, SR, st)
        z = C.nnz
        del C, Afull
        torch.cuda.synchronize()
        phases["allgather_ms"] = phases.get("allgather_ms", 0) + 1e3 * (tb - ta)
        phases["local_ms"] = phases.get("local_ms", 0) + 1e3 * (time.perf_counter() - tb)
        return st.get("multiplies", 0), z

    for _ in range(max(args.warmup, 1)):
        step()
    phases.clear()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    mults = nnzc = 0
    for _ in range(args.steps):
        m, z = step()
        mults += m
        nnzc += z
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=cd)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    s = torch.tensor([mults, nnzc], dtype=torch.float64, device=cd)
    dist.all_reduce(s)
    elapsed, mults, nnzc = float(t.item()), float(s[0].item()), float(s[1].item())
    if rank == 0:
        cfg = workload(args.scale, args.edgefactor, f"1D column split over {world} ranks, A replicated by an "
                       f"all-gather ({backend}); SURVEY 8(e) comparison, not the mandated layout")
        nnza = sum(nzs)
        cfg.update({"nnz_A": nnza, "multiplies": int(mults / args.steps), "nnz_C": int(nnzc / args.steps)})
        print(json.dumps({"metric": METRIC, "value": mults / elapsed, "unit": "multiplies/s", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1000.0 * elapsed / args.steps,
                          "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
                          "data": "synthetic", "config": cfg,
                          "effective_GBps": balg_bytes(mults / args.steps, nnzc / args.steps, nnza, n)
                          / (elapsed / args.steps) / 1e9,
                          "rank0_phases_per_step": {k: round(v / args.steps, 3) for k, v in phases.items()},
                          "input": {"rank0_device_build_s": round(build_s, 4)}}), flush=True)
    dist.destroy_process_group()


# ------------------------------------------------------------------------- rank share (one GPU)
def _hcat(blocks):
    """Blocks side by side (the panel of a grid row: A pieces in stage order)."""
    import torch
    from combblas_amd import dist as cbd
    cps, off = [blocks[0].cp[:1]], 0
    for b in blocks:
        cps.append(b.cp[1:] + off)
        off += b.nnz
    return cbd.Block(blocks[0].nrow, sum(b.ncol for b in blocks), torch.cat(cps), torch.cat([b.ir for b in blocks]),
                     torch.cat([b.val for b in blocks]))


def _vstack(blocks):
    """Blocks stacked by rows (the panel of a grid column: B pieces in stage order), rows ascending per column."""
    import torch
    from combblas_amd import dist as cbd
    ncol, dev = blocks[0].ncol, blocks[0].cp.device
    keys, irs, vals, roff = [], [], [], 0
    for b in blocks:
        col = torch.repeat_interleave(torch.arange(ncol, device=dev), torch.diff(b.cp))
        keys.append(col)
        irs.append(b.ir + roff)
        vals.append(b.val)
        roff += b.nrow
    key = torch.cat(keys)
    order = torch.sort(key, stable=True).indices
    cnt = torch.bincount(key, minlength=ncol)
    cp = torch.zeros(ncol + 1, dtype=torch.int64, device=dev)
    torch.cumsum(cnt, 0, out=cp[1:])
    return cbd.Block(roff, ncol, cp, torch.cat(irs)[order].contiguous(), torch.cat(vals)[order].contiguous())


def _col_slice_block(b, c0, c1):
    import torch
    from combblas_amd import dist as cbd
    lo, hi = int(b.cp[c0].item()), int(b.cp[c1].item())
    return cbd.Block(b.nrow, c1 - c0, (b.cp[c0:c1 + 1] - lo).contiguous(), b.ir[lo:hi], b.val[lo:hi])


def _vlen(x):
    """LEB128 varint bytes of non-negative integers (grid.hip vlen32)."""
    import torch
    return 1 + (x >= 1 << 7).long() + (x >= 1 << 14).long() + (x >= 1 << 21).long() + (x >= 1 << 28).long()


def fiber_wire_bytes(P, chunk=1 << 28):
    """Bytes the fiber pipeline (grid.hip fiber_pipeline) puts on the link for partial P, choosing per message as
    k_code_count's totals do: per-column headers (8 B), rows as varint gaps, 16-bit gaps + 4 B per escaped row (gap >
    65534) or int32, values as varint integers (+8 B per column), u16, f32 or f64 -- the smallest lossless form."""
    import torch
    n, nc = P.nnz, P.ncol
    if n == 0:
        return {"nnz": 0, "bytes": 8 * nc}
    if n > chunk and nc > 1:   # column chunks of ~`chunk` entries: bounded temporaries
        cp_h = P.cp.cpu().numpy()
        import numpy as np
        cuts = [0]
        while cuts[-1] < nc:
            c = int(np.searchsorted(cp_h, cp_h[cuts[-1]] + chunk, side="right")) - 1
            cuts.append(min(nc, max(c, cuts[-1] + 1)))
        parts = [fiber_wire_bytes(_col_slice_block(P, a, b), chunk) for a, b in zip(cuts[:-1], cuts[1:])]
        rows = {k: sum(p["row_bytes"].get(k, 0) for p in parts if p["nnz"]) for k in ("int32", "gap16", "varint")}
        vals = {"f64": 8 * n}
        for k in ("f32", "u16", "varint"):
            if all(k in p["value_bytes"] for p in parts if p["nnz"]):
                vals[k] = sum(p["value_bytes"][k] for p in parts if p["nnz"])
        rf, vf = min(rows, key=rows.get), min(vals, key=vals.get)
        return {"nnz": n, "escapes": sum(p.get("escapes", 0) for p in parts), "rows": rf, "values": vf,
                "row_bytes": rows, "value_bytes": vals, "bytes": 8 * nc + rows[rf] + vals[vf],
                "bytes_per_entry": round((8 * nc + rows[rf] + vals[vf]) / n, 3)}
    cnt = torch.diff(P.cp)
    starts = P.cp[:-1][cnt > 0]
    ir = P.ir.to(torch.int64)
    prev = torch.roll(ir, 1)
    prev[starts] = 0
    gap = ir - prev
    esc = int((gap > 0xFFFE).sum().item())
    rows = {"int32": 4 * n, "gap16": 2 * n + 4 * esc, "varint": int(_vlen(gap).sum().item())}
    v = P.val
    vals = {"f64": 8 * n}
    if bool((v.to(torch.float32).to(torch.float64) == v).all().item()):
        vals["f32"] = 4 * n
    is_int = (v == torch.round(v)) & (v >= 0)
    if bool((is_int & (v <= 65535)).all().item()):
        vals["u16"] = 2 * n
    if bool((is_int & (v <= 4294967295.0)).all().item()):
        vals["varint"] = int(_vlen(v.to(torch.int64)).sum().item()) + 8 * nc
    rf = min(rows, key=rows.get)
    vf = min(vals, key=vals.get)
    return {"nnz": n, "escapes": esc, "rows": rf, "values": vf, "row_bytes": rows, "value_bytes": vals,
            "bytes": 8 * nc + rows[rf] + vals[vf], "bytes_per_entry": round((8 * nc + rows[rf] + vals[vf]) / n, 3)}


def bench_rank_share(args):
    """One rank's share of the N-GPU product, on this one GPU, without a transport: rank (l, i, j) of the
    mandated layout builds its panels (A's grid row i and B's grid column j over layer l's inner range: what the
    panel schedule's broadcasts deliver), multiplies the other layer's column half, measures the fiber message that
    half would make, multiplies its own half, and merges it with the partner's message (the partner rank's product
    of this rank's half, computed here beforehand).  Records local ms, fiber bytes and the peak HBM in use."""
    import tempfile
    import torch
    import torch.distributed as dist
    import combblas_amd as cb
    from combblas_amd import dist as cbd
    N = args.gpus_virtual
    L, q, _ = cbd.grid_for(N)
    ranks = list(range(N)) if args.rank_share == "all" else [int(x) for x in args.rank_share.split(",")]
    store = tempfile.NamedTemporaryFile(delete=False)
    dist.init_process_group("gloo", init_method=f"file://{store.name}", rank=0, world_size=1)
    ctx = cb.Context(0)
    be = cbd.GpuBackend(ctx)
    SR = cb.PlusTimesSRing("f64")
    n = 1 << args.scale
    dev = be.device
    total = torch.cuda.mem_get_info()[1]
    floor = [total]

    def sample():
        torch.cuda.synchronize()
        floor[0] = min(floor[0], torch.cuda.mem_get_info()[0])

    def panels(l, i, j, c0=None, c1=None):
        r0, r1 = cbd.block_range(n, q, i)
        k_ranges = [cbd.piece_range(n, q, L, k, l) for k in range(q)]
        b0, b1 = cbd.block_range(n, q, j)
        AP = _hcat([be.rmat_block(args.scale, args.edgefactor, args.seed, r0, r1, k0, k1) for (k0, k1) in k_ranges])
        BP = _vstack([be.rmat_block(args.scale, args.edgefactor, args.seed, k0, k1, b0, b1) for (k0, k1) in k_ranges])
        return AP, BP

    bad = False
    for r in ranks:
        l, rem = divmod(r, q * q)
        i, j = divmod(rem, q)
        t0 = time.perf_counter()
        AP, BP = panels(l, i, j)
        nc = BP.ncol
        halves = [cbd.block_range(nc, L, m) for m in range(L)]
        me, other = (l, 1 - l) if L == 2 else (0, None)
        build_s = time.perf_counter() - t0
        rec = {"rank": r, "layout": f"{L}x{q}x{q}", "l_i_j": [l, i, j], "scale": args.scale,
               "nnz_A_panel": AP.nnz, "nnz_B_panel": BP.nnz, "panel_build_s": round(build_s, 3)}
        torch.cuda.empty_cache()
        sample()

        def partner_piece():
            """The partner's message: its product of this rank's column half (made after the own half, as it
            arrives in the pipeline, so it is not held during this rank's products)."""
            PA, PB = panels(other, i, j)
            P = be.multiply(PA, _col_slice_block(PB, *halves[me]), SR)
            del PA, PB
            return P

        phase_keys = ("flops_ms", "bin_ms", "symbolic_ms", "scan_ms", "numeric_ms", "heavy_ms", "total_ms")
        gather = L == 2 and args.fiber_mode == "gather"
        if gather:   # the fiber gather (grid.hip fiber_gather): the partner's operands, as they would arrive
            PA, PB = panels(other, i, j)
            mine_b = _col_slice_block(BP, *halves[me])
            sent_b = _col_slice_block(BP, *halves[other])
            ent = 4 + 8   # row + f64 value
            rec["gather_bytes_sent"] = AP.nnz * ent + 8 * (AP.ncol + 1) + sent_b.nnz * ent + 8 * (sent_b.ncol + 1)
            part_b = _col_slice_block(PB, *halves[me])
            rec["gather_bytes_recv"] = PA.nnz * ent + 8 * (PA.ncol + 1) + part_b.nnz * ent + 8 * (part_b.ncol + 1)
            A2 = _hcat([AP, PA] if me == 0 else [PA, AP])
            B2 = _vstack([mine_b, part_b] if me == 0 else [part_b, mine_b])
            del PA, PB, mine_b, sent_b, part_b
            torch.cuda.empty_cache()
        for rep in range(2):   # the second repetition is recorded (code objects loaded, pool warm)
            floor[0] = torch.cuda.mem_get_info()[0]
            st = {}
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if gather:
                Pm = be.multiply(A2, B2, SR, st)
                sample()
                local_ms = 1e3 * (time.perf_counter() - t0)
                merge_ms, wire = 0.0, None
                nnz_out = Pm.nnz
                profs = [ctx.last_profile()]
                final = Pm if rep == 1 else None
                del Pm
            elif L == 2:
                Po = be.multiply(AP, _col_slice_block(BP, *halves[other]), SR, st)
                sample()
                t1 = time.perf_counter()
                p_other = ctx.last_profile()
                wire = fiber_wire_bytes(Po)
                if rep == 1:   # the production encoder + decoder on the same message (cbg_fiber_codec)
                    chunks = int(os.environ.get("CBG_FIBER_CHUNKS", "2"))
                    codec = be.fiber_codec(Po, chunks)
                del Po
                t2 = time.perf_counter()
                Pm = be.multiply(AP, _col_slice_block(BP, *halves[me]), SR, st)
                sample()
                t3 = time.perf_counter()
                p_mine = ctx.last_profile()
                Pr = partner_piece()
                rec["recv_nnz"] = Pr.nnz
                torch.cuda.synchronize()
                t4 = time.perf_counter()
                M = be.merge([Pm, Pr] if me == 0 else [Pr, Pm], SR)
                sample()
                t5 = time.perf_counter()
                local_ms = 1e3 * ((t1 - t0) + (t3 - t2))
                merge_ms = 1e3 * (t5 - t4)
                nnz_out = M.nnz
                final = M if rep == 1 else None   # checked below, after the record's timings
                del Pm, M, Pr
                profs = [p_other, p_mine]
            else:
                Pm = be.multiply(AP, BP, SR, st)
                sample()
                local_ms = 1e3 * (time.perf_counter() - t0)
                merge_ms, wire = 0.0, None
                nnz_out = Pm.nnz
                profs = [ctx.last_profile()]
                final = Pm if rep == 1 else None
                del Pm
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
        del AP, BP
        if gather:
            del A2, B2
        torch.cuda.empty_cache()
        # the rank's finished piece C(rows_i, columns) against its independent reference (verify_piece)
        r0, r1 = cbd.block_range(n, q, i)
        b0, _ = cbd.block_range(n, q, j)
        h0, h1 = halves[me]
        Arow, Acol, est_m, est_z = piece_reference(be, args, n, r0, r1, b0 + h0, b0 + h1)
        nsample = max(int(np.ceil(1e4 / N)), final.ncol // 64)
        v = verify_piece(be, SR, final, Arow, Acol, r0, b0 + h0, nsample, args.seed + 7919 * r,
                         oracle_cols=0 if args.no_cpu else 256)
        v.update({"piece_nnz": final.nnz, "piece_nnz_equals_estimate": final.nnz == est_z,
                  "piece_multiplies_estimate": est_m})
        rec["verified"] = v
        rec["fiber_mode"] = "gather" if gather else ("reduce" if L == 2 else "none")
        if L == 2 and not gather:
            rec["fiber_codec"] = codec
            rec["fiber_codec_vs_estimate"] = round(codec["wire_bytes"] / max(wire["bytes"], 1), 5)
        del final, Arow, Acol
        torch.cuda.empty_cache()
        rec["phases_ms"] = [{k: round(float(pp[k]), 3) for k in phase_keys} for pp in profs]
        # what the heavy kernels processed per product (cbg_profile): the rank's heavy roofline
        rec["heavy_counts"] = [{k: int(pp.get(k, 0)) for k in ("heavy_multiplies", "heavy_nnz_b", "heavy_nnz_c")}
                               for pp in profs]
        hb = sum(c["heavy_multiplies"] * (S_I + S_V) + c["heavy_nnz_b"] * (S_I + S_V + 2 * S_P)
                 + c["heavy_nnz_c"] * (S_I + S_V) for c in rec["heavy_counts"])
        hms = sum(float(pp["heavy_ms"]) for pp in profs)
        rec["heavy_GBps"] = round(hb / (hms / 1e3) / 1e9, 1) if hms > 0 else None
        rec.update({"multiplies": st.get("multiplies", 0), "local_ms": round(local_ms, 3),
                    "merge_ms": round(merge_ms, 3), "nnz_C_piece": nnz_out,
                    "heavy_ms": round(sum(p["heavy_ms"] for p in profs), 3),
                    "symbolic_ms": round(sum(p["symbolic_ms"] for p in profs), 3),
                    "fiber": wire,
                    "peak_hbm_GB": round((total - floor[0]) / 1e9, 2), "hbm_total_GB": round(total / 1e9, 1)})
        print(json.dumps(rec), flush=True)
        bad = bad or not (v["bit_exact"] and v["piece_nnz_equals_estimate"]
                          and (L == 1 or gather or codec["roundtrip_exact"]))
    dist.destroy_process_group()
    if os.path.exists(store.name):
        os.unlink(store.name)
    if bad:
        sys.exit("bench: a rank's piece failed its checks (verified / fiber_codec)")


# ------------------------------------------------------------------------- rank launcher (N > 1)
def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _visible_device_count():
    """GPUs this process could use, counted without initialising the GPU (torch.cuda.device_count() does not on
    this ROCm image; the environment's visibility masks are honoured by it)."""
    try:
        import torch
        return torch.cuda.device_count()
    except Exception:
        return 0


def launch_ranks(n, argv, grace_s=30.0):
    """`bench.py --gpus N` without WORLD_SIZE: start N fresh child processes of this script, one per GPU, BEFORE any
    GPU call in this process (the parent only counts devices), as torch.distributed.run would: RANK = LOCAL_RANK = r,
    WORLD_SIZE = LOCAL_WORLD_SIZE = N, MASTER_ADDR 127.0.0.1 and a free port.  Rank 0's stdout is this process's
    stdout (its one JSON line); the other ranks' stdout goes to stderr.  When a rank fails, the others get `grace_s`
    to finish (they would otherwise wait in a collective for the dead rank), then SIGTERM, then SIGKILL -- each by
    its own PID.  Returns the exit status: 0 only if every rank exited 0.  The reference's driver likewise sizes its
    grid from the launched world (3DSpGEMM/mpipspgemm.cpp:34-60)."""
    import signal
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno(), text=True))

    def relay(stream):   # rank 0's JSON line to stdout; library chatter (gloo/RCCL banners) to stderr
        for line in stream:
            out = sys.stdout if line.startswith("{") else sys.stderr
            out.write(line)
            out.flush()
    import threading
    relay_thread = threading.Thread(target=relay, args=(procs[0].stdout,), daemon=True)
    relay_thread.start()

    def forward(signum, _frame):   # the launcher stopped (e.g. a time limit): stop every rank it started
        for p in procs:
            if p.poll() is None:
                p.send_signal(signum)
        for p in procs:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                p.kill()
        sys.exit(128 + signum)
    signal.signal(signal.SIGTERM, forward)
    signal.signal(signal.SIGINT, forward)
    status = 0
    failed_at = None
    while True:
        codes = [p.poll() for p in procs]
        for r, c in enumerate(codes):
            if c not in (None, 0) and status == 0:
                status = c if c > 0 else 128 - c
                failed_at = time.monotonic()
                print(f"bench: rank {r} exited with status {c}", file=sys.stderr, flush=True)
        if all(c is not None for c in codes):
            break
        if failed_at is not None and time.monotonic() - failed_at > grace_s:
            for p in procs:
                if p.poll() is None:
                    p.send_signal(signal.SIGTERM)
            t = time.monotonic()
            while any(p.poll() is None for p in procs) and time.monotonic() - t < 10:
                time.sleep(0.2)
            for p in procs:
                if p.poll() is None:
                    p.kill()
            for p in procs:
                p.wait()
            break
        time.sleep(0.2)
    relay_thread.join(timeout=10)
    return status


def launch_probe(world, rank, local_rank):
    """`--launch-probe` (launcher test, CPU): every rank joins a gloo group and rank 0 prints the line the launched
    world produced -- the same rendezvous and one-line contract as the real run, without a GPU."""
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    recs = [None] * world
    dist.all_gather_object(recs, {"rank": rank, "local_rank": local_rank, "pid": os.getpid(),
                                  "world": int(os.environ["WORLD_SIZE"])})
    t = torch.tensor([float(rank)])
    dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "n_gpus": world, "launch_probe": True, "world": dist.get_world_size(),
                          "rank_sum": float(t.item()), "ranks": recs}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    if os.environ.get("CBG_LAUNCH_PROBE_FAIL_RANK") == str(rank):
        sys.exit(7)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks); default WORLD_SIZE or 1.  Without WORLD_SIZE, N > 1 starts N ranks itself")
    ap.add_argument("--launch-probe", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--scale", type=int, default=0, help="R-MAT scale (default 20 + {1:0,2:1,4:1,8:2}[N])")
    ap.add_argument("--edgefactor", type=int, default=16)
    ap.add_argument("--seed", type=int, default=0xDECAFBAD, help="Graph500 user seed (the reference's SEED)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--layout", choices=["3d", "1d"], default="3d",
                    help="N > 1: the mandated 1x1x2 / 2x2 / 2x2x2 layouts (default) or SURVEY 8(e)'s 1D comparison")
    ap.add_argument("--cpu-mults", type=float, default=1.5e9, help="multiplies in the CPU baseline sample")
    ap.add_argument("--rank-share", default=None,
                    help="with --gpus-virtual N: run these ranks' shares of the N-GPU layout on this one GPU "
                         "('all' or a comma list); one JSON line per rank (local ms, fiber bytes, peak HBM)")
    ap.add_argument("--gpus-virtual", type=int, default=8)
    ap.add_argument("--fiber-mode", choices=["gather", "reduce"], default="gather",
                    help="--rank-share on two-layer layouts: the fiber gather of the operands (what the grid takes for "
                         "A*A) or the reduction of partial products (codec + merge)")
    args = ap.parse_args()
    if args.rank_share is None and "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        # launched as `python bench.py --gpus N`: this process becomes the launcher; it makes no GPU call
        backend = os.environ.get("CBG_DIST_BACKEND", "nccl")
        have = _visible_device_count()
        if not args.launch_probe and backend == "nccl" and have < args.gpus:
            sys.exit(f"bench: --gpus {args.gpus} needs {args.gpus} visible GPUs for RCCL (found {have}); a rehearsal "
                     f"with ranks sharing GPUs sets CBG_DIST_BACKEND=rccl-net or gloo")
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is not None and args.rank_share is None and args.gpus != world:
        sys.exit(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}: the launched world must match")
    args.gpus = world
    if args.launch_probe:
        return launch_probe(world, rank, local_rank)
    if args.rank_share is not None:
        if not args.scale:
            args.scale = 20 + {1: 0, 2: 1, 4: 1, 8: 2}.get(args.gpus_virtual, 0)
        return bench_rank_share(args)
    if not args.scale:
        args.scale = 20 + {1: 0, 2: 1, 4: 1, 8: 2}.get(world, 0)
    if world == 1:
        bench_local(args)
    else:
        bench_dist(args, world, rank, local_rank)


if __name__ == "__main__":
    main()
