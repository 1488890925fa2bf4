#!/usr/bin/env python3
"""Benchmark: SpGEMM multiplies/s on R-MAT A*A (PlusTimes<double>), MI355X-native local hash SpGEMM.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scale S] [--no-cpu]

One "step" = one full local SpGEMM C = A*B through the C ABI (column stats, binning, symbolic,
scan, allocation of C, numeric with row-sorted output), inputs already resident in HBM.

N = 1: the whole product on one GPU (BASELINE config 2: R-MAT scale-20, edge factor 16).
N > 1 (torchrun, one rank per GPU): A is generated identically on every rank (deterministic seed),
B's columns are split into N contiguous ranges of equal multiplies, and each rank computes its
C(:, range) -- independent output columns, no data-path collective ("replicas of A").  Total work is
fixed (strong scaling).  Timing: barrier + device sync around exactly K steps, max over ranks.

Prints ONE JSON line on rank 0 (schema in the task contract) with `roofline` for the numeric phase and
`cpu_baseline` = the oracle CPU restatement timed on a bounded sample of the same product.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
S_I, S_V, S_P = 4, 8, 8        # row-index, value, column-pointer bytes


def balg_bytes(mults, nnzc, nnzb, ncolb):
    """SURVEY §8(d) algorithmic bytes of one whole SpGEMM."""
    return (mults * (2 * S_I + S_V) + nnzc * (S_I + S_V) + nnzb * (2 * S_I + S_V + 4 * S_P)
            + 4 * (ncolb + 1) * S_P)


def numeric_bytes(mults, nnzc, nnzb, ncolb):
    """Algorithmic bytes of the numeric phase only (the dominant kernels): gather A (row,val) per
    multiply, read B (row,val) + A colptr pair per B nonzero, write C (row,val), colptr."""
    return mults * (S_I + S_V) + nnzb * (S_I + S_V + 2 * S_P) + nnzc * (S_I + S_V) + 2 * (ncolb + 1) * S_P


def flop_split(cp, ir, nparts):
    """Column ranges of equal multiplies (estimateFLOP per column, mtSpGEMM.h:1117-1135)."""
    nnz_col = np.diff(cp)
    per_b = nnz_col[ir]                      # nnz(A(:,k)) for every B nonzero (B = A)
    csum = np.concatenate([[0], np.cumsum(per_b)])
    flop_col = csum[cp[1:]] - csum[cp[:-1]]
    cum = np.cumsum(flop_col)
    tot = cum[-1]
    bounds = [0]
    for r in range(1, nparts):
        bounds.append(int(np.searchsorted(cum, tot * r / nparts)))
    bounds.append(len(flop_col))
    return bounds, flop_col


def cpu_baseline(cp, ir, val, n, flop_col, target_mults):
    """Oracle (CPU restatement, oracle/oracle.c) on a bounded sample: every s-th column of B."""
    sys.path.insert(0, os.path.join(HERE, "tests"))
    from helpers import Csc, oracle_spgemm  # test infrastructure: checker/baseline only
    tot = int(flop_col.sum())
    stride = max(1, int(np.ceil(tot / max(target_mults, 1))))
    cols = np.arange(0, n, stride)
    bcp = np.concatenate([[0], np.cumsum(np.diff(cp)[cols])]).astype(np.int64)
    idx = np.concatenate([np.arange(cp[c], cp[c + 1]) for c in cols]) if len(cols) else np.zeros(0, np.int64)
    A = Csc(n, n, cp, ir, val)
    B = Csc(n, len(cols), bcp, ir[idx], val[idx])
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    t0 = time.perf_counter()
    C, mults, rc = oracle_spgemm(A, B, "plus_times", "f64")
    dt = time.perf_counter() - t0
    assert rc == 0
    return {"value": mults / dt, "unit": "multiplies/s", "cores": threads, "kind": "port",
            "sample": f"oracle/oracle.c (CPU restatement of LocalSpGEMMHash, OpenMP) on every {stride}-th "
                      f"column of B ({len(cols)} columns, {mults} multiplies, {dt:.2f} s)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--scale", type=int, default=20)
    ap.add_argument("--edgefactor", type=int, default=16)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-mults", type=float, default=1.5e9, help="multiplies in the CPU baseline sample")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl" if torch.cuda.is_available() else "gloo")

    import combblas_amd as cb
    from combblas_amd import _abi

    n, cp, ir, val = cb.generate_rmat_host(args.scale, args.edgefactor, seed=args.seed)
    bounds, flop_col = flop_split(cp, ir, world)
    c0, c1 = bounds[rank], bounds[rank + 1]

    ctx = cb.Context(local_rank if world > 1 else 0)
    A = cb.SpDCCols.from_csc(ctx, n, n, cp, ir, val)
    va = A._view()
    vb = A._view()
    # B = A(:, c0:c1): same device arrays, colptr offset (absolute positions stay valid)
    vb.ncol = c1 - c0
    vb.nzc = c1 - c0
    vb.cp = (va.cp or 0) + 8 * c0
    vb.nnz = int(cp[c1] - cp[c0])

    import ctypes
    lib = ctx._lib

    def step():
        res = _abi.CscResult()
        m = ctypes.c_int64()
        _abi.check(lib.cbg_spgemm_local(ctx._ptr, ctypes.byref(va), ctypes.byref(vb), _abi.SR_PLUS_TIMES,
                                        _abi.F64, _abi.SORTED_COLS, ctypes.byref(res), ctypes.byref(m)),
                   "cbg_spgemm_local")
        prof = ctx.last_profile()
        nnzc = int(res.nnz)
        lib.cbg_result_free(ctx._ptr, ctypes.byref(res))
        return int(m.value), nnzc, prof

    def barrier():
        ctx.synchronize()
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    barrier()
    t0 = time.perf_counter()
    mults = nnzc = 0
    num_ms = []
    tot_ms = []
    for _ in range(args.steps):
        m, z, prof = step()
        mults += m
        nnzc += z
        num_ms.append(prof["numeric_ms"])
        tot_ms.append(prof["total_ms"])
    barrier()
    elapsed = time.perf_counter() - t0

    local = np.array([elapsed, mults, nnzc, np.mean(num_ms)], np.float64)
    if dist is not None:
        import torch
        t = torch.tensor(local, dtype=torch.float64, device="cuda")
        tmax = t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tsum = t.clone()
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        elapsed, mults, nnzc = float(tmax[0]), float(tsum[1]), float(tsum[2])
        num_mean_ms = float(tmax[3])
    else:
        num_mean_ms = float(np.mean(num_ms))

    if rank == 0:
        ms_per_step = 1000.0 * elapsed / args.steps
        mult_step = mults / args.steps
        nnzc_step = nnzc / args.steps
        value = mults / elapsed
        nnzb = int(cp[-1])
        b_alg = balg_bytes(mult_step, nnzc_step, nnzb, n)
        nb = numeric_bytes(mult_step / world, nnzc_step / world, nnzb / world, n / world)
        achieved = nb / (num_mean_ms / 1e3) / 1e9
        out = {
            "metric": "SpGEMM multiplies/sec, R-MAT s22 A·A at 1/2/4/8 MI355X + achieved HBM GB/s",
            "value": value, "unit": "multiplies/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": f"R-MAT (Graph500 Kronecker, clip-and-flip, scrambled) scale-{args.scale} "
                                   f"edge factor {args.edgefactor} A*A PlusTimes<double>, local hash SpGEMM "
                                   f"(BASELINE config 2)",
                       "scale": args.scale, "edgefactor": args.edgefactor, "nnz_A": nnzb,
                       "multiplies": int(mult_step), "nnz_C": int(nnzc_step),
                       "parallelism": "single" if world == 1 else f"1D column split x{world}, A replicated"},
            "effective_GBps": b_alg / (elapsed / args.steps) / 1e9,
            "roofline": {"bound": "hbm", "kernel": "numeric phase (k_num_wave/k_num_block/k_window)",
                         "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": None},
        }
        if world == 1 and not args.no_cpu:
            out["cpu_baseline"] = cpu_baseline(cp, ir, val, n, flop_col, args.cpu_mults)
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
