#!/usr/bin/env python3
"""Can an RCCL-sized kernel start while the SpGEMM runs?  (diagnostic, not a test)

RCCL's device kernel on gfx950 (ncclDevKernel_Generic) is a 512-thread workgroup with 37,664 B of static LDS
(llvm-readelf --notes of librccl.so's gfx950 code object).  k_num_heavy_known is a persistent grid of one
1024-thread workgroup per CU holding ~152.7 KB of the CU's 160 KB of LDS.  This probe runs R-MAT products back to
back on the library's stream while a second host thread launches tools/probe/liblds_copy.so's copy kernel (RCCL's
footprint: 512 threads, 37,664 B LDS, `--wg` workgroups) on another stream at random moments, one launch at a time,
and records per launch the time from the stream reaching the launch to the copy's end (HIP events on the copy
stream).  A launch that lands while the heavy grid holds every CU waits for it: its time grows by up to the heavy
kernel's duration.  Also reports the products' heavy-kernel time with and without the concurrent copies (a static
persistent grid whose workgroup is held back by a resident copy stretches the kernel; a ticketed one does not).

usage: python tools/coresidency_probe.py [--scale 20] [--wg 16] [--mb 256] [--seconds 4] [--lib path/libcbgpu.so]
Environment: CBG_HEAVY_RESERVE_CU=k leaves k CUs free of the persistent heavy grids.  Prints one JSON line.
"""
import argparse
import ctypes
import json
import os
import random
import sys
import threading
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=20)
    ap.add_argument("--wg", type=int, default=16)
    ap.add_argument("--mb", type=int, default=256, help="bytes per copy launch (MiB)")
    ap.add_argument("--seconds", type=float, default=4.0)
    ap.add_argument("--lib", default=None)
    ap.add_argument("--tag", default="")
    args = ap.parse_args()
    from combblas_amd import _abi
    if args.lib:
        _abi.LIB_PATH = os.path.abspath(args.lib)
    import torch
    import combblas_amd as cb

    probe = ctypes.CDLL(os.path.join(HERE, "probe", "liblds_copy.so"))
    probe.probe_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int]
    lds = ctypes.c_int(0)
    probe.probe_lds_bytes(ctypes.byref(lds))

    ctx = cb.Context(0)
    A = ctx.generate_rmat(args.scale)
    ctx.synchronize()
    va = A._view()
    lib = ctx._lib
    nbytes = args.mb << 20
    src = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    dst = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    s2 = torch.cuda.Stream()

    def product():
        res = _abi.CscResult()
        m = ctypes.c_int64()
        _abi.check(lib.cbg_spgemm_local(ctx._ptr, ctypes.byref(va), ctypes.byref(va), _abi.SR_PLUS_TIMES, _abi.F64,
                                        _abi.SORTED_COLS, ctypes.byref(res), ctypes.byref(m)), "cbg_spgemm_local")
        p = ctx.last_profile()
        lib.cbg_result_free(ctx._ptr, ctypes.byref(res))
        return p

    def copy_once():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s2)
        rc = probe.probe_copy(ctypes.c_void_p(s2.cuda_stream), ctypes.c_void_p(src.data_ptr()),
                              ctypes.c_void_p(dst.data_ptr()), nbytes, args.wg)
        assert rc == 0, rc
        e1.record(s2)
        e1.synchronize()
        return e0.elapsed_time(e1)

    for _ in range(3):
        product()
    ctx.synchronize()
    alone = [copy_once() for _ in range(20)]
    solo = [product() for _ in range(5)]

    stop = threading.Event()
    times = []

    def copier():
        rnd = random.Random(1)
        while not stop.is_set():
            time.sleep(rnd.uniform(0.0, 0.02))
            times.append(copy_once())

    th = threading.Thread(target=copier)
    th.start()
    busy = []
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < args.seconds:
        busy.append(product())
    stop.set()
    th.join()
    ctx.synchronize()

    med0 = float(np.median(alone))
    t = np.array(times)

    def pct(x, q):
        return round(float(np.percentile(x, q)), 3) if len(x) else None

    out = {"probe": "coresidency", "tag": args.tag, "lib": os.path.relpath(_abi.LIB_PATH, REPO),
           "reserve_cu_env": os.environ.get("CBG_HEAVY_RESERVE_CU", "0"), "scale": args.scale,
           "copy": {"workgroups": args.wg, "threads": 512, "lds_bytes": lds.value, "bytes": nbytes},
           "copy_alone_ms": {"median": round(med0, 3), "max": round(float(np.max(alone)), 3),
                             "GBps": round(nbytes / med0 / 1e6, 1)},
           "copy_during_products_ms": {"n": int(len(t)), "median": pct(t, 50), "p75": pct(t, 75), "p90": pct(t, 90),
                                       "max": pct(t, 100),
                                       "delayed_over_2x": int((t > 2 * med0).sum()),
                                       "delayed_over_10ms": int((t > med0 + 10).sum())},
           "product_solo_ms": {"total": round(float(np.median([p["total_ms"] for p in solo])), 3),
                               "heavy": round(float(np.median([p["heavy_ms"] for p in solo])), 3)},
           "product_with_copies_ms": {"n": len(busy),
                                      "total_median": round(float(np.median([p["total_ms"] for p in busy])), 3),
                                      "heavy_median": round(float(np.median([p["heavy_ms"] for p in busy])), 3),
                                      "heavy_max": round(float(np.max([p["heavy_ms"] for p in busy])), 3)}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
