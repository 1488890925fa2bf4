#!/usr/bin/env python3
"""Overlap probe for the fiber pipeline on ONE GPU: does the fiber codec (k_code_count / k_var_encode / k_var_decode,
one-wave workgroups) run beside a rank's own-half product, and what does each cost the other?

Rank (l, i, j) of the N-GPU layout (bench.py --rank-share's panels, R-MAT scale s): the other layer's column half is
multiplied once to make the message; then, each three times:
  alone     the own-half product (library context 1, its stream)          -> product_ms
  alone     cbg_fiber_codec on the message (context 2, its own stream)    -> codec_ms (encode + decode, C chunks)
  together  both at once from two host threads (ctypes drops the GIL)      -> wall_ms, product_ms, codec_ms
The fiber pipeline decodes each received chunk on a decode stream while the own columns multiply (grid.hip); this
measures that concurrency on the hardware without a second GPU.  One JSON line.
usage: python tools/overlap_probe.py [--scale 22] [--gpus-virtual 8] [--rank 0] [--chunks 2] [--reps 3]"""
import argparse
import json
import os
import sys
import tempfile
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=22)
    ap.add_argument("--gpus-virtual", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--chunks", type=int, default=2)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import numpy as np
    import torch
    import torch.distributed as dist
    import combblas_amd as cb
    from combblas_amd import dist as cbd
    import bench

    store = tempfile.NamedTemporaryFile(delete=False)
    dist.init_process_group("gloo", init_method=f"file://{store.name}", rank=0, world_size=1)
    ctx1, ctx2 = cb.Context(0), cb.Context(0)
    be1, be2 = cbd.GpuBackend(ctx1), cbd.GpuBackend(ctx2)
    SR = cb.PlusTimesSRing("f64")
    N, s = args.gpus_virtual, args.scale
    n = 1 << s
    L, q, _ = cbd.grid_for(N)
    if L != 2:
        sys.exit("overlap_probe: the layout has no fiber exchange (use 2 or 8 virtual GPUs)")
    l, rem = divmod(args.rank, q * q)
    i, j = divmod(rem, q)
    seed = cb.G500_SEED

    def panels(layer):
        r0, r1 = cbd.block_range(n, q, i)
        b0, b1 = cbd.block_range(n, q, j)
        kr = [cbd.piece_range(n, q, L, k, layer) for k in range(q)]
        AP = bench._hcat([be1.rmat_block(s, 16, seed, r0, r1, k0, k1) for (k0, k1) in kr])
        BP = bench._vstack([be1.rmat_block(s, 16, seed, k0, k1, b0, b1) for (k0, k1) in kr])
        return AP, BP

    AP, BP = panels(l)
    halves = [cbd.block_range(BP.ncol, L, m) for m in range(L)]
    mine, other = halves[l], halves[1 - l]
    Bmine = bench._col_slice_block(BP, *mine)
    msg = be1.multiply(AP, bench._col_slice_block(BP, *other), SR)   # the message this rank sends
    torch.cuda.synchronize()

    def product():
        t0 = time.perf_counter()
        P = be1.multiply(AP, Bmine, SR)
        ctx1.synchronize()
        dt = time.perf_counter() - t0
        del P
        return 1e3 * dt

    def codec():
        t0 = time.perf_counter()
        st = be2.fiber_codec(msg, args.chunks)
        ctx2.synchronize()
        return 1e3 * (time.perf_counter() - t0), st

    product()
    codec()   # warm-up: code objects, pools
    torch.cuda.synchronize()
    alone_p, alone_c, tog = [], [], []
    last = None
    for _ in range(args.reps):
        alone_p.append(product())
        torch.cuda.synchronize()
        c_ms, last = codec()
        alone_c.append((c_ms, last["encode_ms"], last["decode_ms"]))
        torch.cuda.synchronize()
        out = {}

        def run_p():
            out["p"] = product()

        def run_c():
            out["c"] = codec()
        t0 = time.perf_counter()
        ths = [threading.Thread(target=run_p), threading.Thread(target=run_c)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        wall = 1e3 * (time.perf_counter() - t0)
        tog.append((wall, out["p"], out["c"][0], out["c"][1]["roundtrip_exact"]))
        torch.cuda.synchronize()
    med = lambda xs: float(np.median(xs))
    rec = {"probe": "own-half product || fiber codec (two contexts, two streams, one GPU)",
           "layout": f"{L}x{q}x{q}", "rank": args.rank, "scale": s, "chunks": args.chunks,
           "message_entries": msg.nnz, "wire_bytes": last["wire_bytes"],
           "alone": {"product_ms": round(med(alone_p), 3), "codec_ms": round(med([x[0] for x in alone_c]), 3),
                     "encode_ms": round(med([x[1] for x in alone_c]), 3),
                     "decode_ms": round(med([x[2] for x in alone_c]), 3)},
           "together": {"wall_ms": round(med([x[0] for x in tog]), 3), "product_ms": round(med([x[1] for x in tog]), 3),
                        "codec_ms": round(med([x[2] for x in tog]), 3)},
           "roundtrip_exact": all(bool(x[3]) for x in tog) and bool(last["roundtrip_exact"])}
    a, t = rec["alone"], rec["together"]
    rec["hidden_ms"] = round(a["product_ms"] + a["codec_ms"] - t["wall_ms"], 3)
    rec["hidden_frac_of_codec"] = round(rec["hidden_ms"] / max(a["codec_ms"], 1e-9), 3)
    print(json.dumps(rec), flush=True)
    dist.destroy_process_group()
    if os.path.exists(store.name):
        os.unlink(store.name)
    if not rec["roundtrip_exact"]:
        sys.exit("overlap_probe: the codec round trip differs")


if __name__ == "__main__":
    main()
