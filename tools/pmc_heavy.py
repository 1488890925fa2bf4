#!/usr/bin/env python3
"""HBM traffic of the heavy-column numeric phase (k_num_heavy_known + k_num_heavy, the kernels between
the heavy_ms events) from rocprofv3 PMC passes -> profiles/<tag>_pmc_heavy.json.

Run on the GPU box (each counter group is its own rocprofv3 run, MI355X_MICROARCH.md §rocprofv3):
    python tools/pmc_heavy.py run <tag> [scale]      # two PMC passes over bench.py + summary
    python tools/pmc_heavy.py product <tag> [scale]  # whole-product traffic (four passes)
FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (TCC EA requests).  The guide's gfx950 correction
(FETCH_SIZE reads 1/2 of a 16-B-per-lane coalesced stream) is calibrated for wide streaming loads
only; k_num_heavy's loads are 4/8-B gathers plus 16-B segment reads, so the JSON carries the raw
counter sum as `bytes_per_launch` and the doubled-fetch figure as an upper bound beside it.
"""
import csv
import glob
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def per_dispatch(path, kernel_substr):
    vals = {}
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel_substr in r["Kernel_Name"]:
                key = (r["Dispatch_Id"], r["Counter_Name"])
                vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    out = {}
    for (d, c), v in vals.items():
        out.setdefault(c, []).append(v)
    return out


def run(tag, scale):
    out = os.path.join(REPO, "gpurun_out", tag)
    os.makedirs(out, exist_ok=True)
    env = dict(os.environ, TMPDIR="/tmp")
    for i, ctr in enumerate(("FETCH_SIZE", "WRITE_SIZE")):
        cmd = ["timeout", "-s", "KILL", "240", "rocprofv3", "--pmc", ctr, "--output-format", "csv",
               "-d", os.path.join(out, f"pmc{i}"), "-o", "run", "--", sys.executable, os.path.join(REPO, "bench.py"),
               "--steps", "1", "--warmup", "1", "--no-cpu", "--scale", str(scale)]
        r = subprocess.run(cmd, env=env, cwd=REPO, stdout=open(os.path.join(out, f"pmc{i}.log"), "w"),
                           stderr=subprocess.STDOUT)
        print(f"pass {ctr}: rc={r.returncode}", flush=True)
        if r.returncode != 0:
            sys.exit(r.returncode)
    nprod = 2   # --warmup 1 --steps 1: two products; every product launches each heavy kernel once
    f = per_dispatch(os.path.join(out, "pmc0"), "k_num_heavy").get("FETCH_SIZE", [])
    w = per_dispatch(os.path.join(out, "pmc1"), "k_num_heavy").get("WRITE_SIZE", [])
    if not f or not w:
        sys.exit("no k_num_heavy dispatches in the PMC output")
    fetch = sum(f) / nprod * 1024.0
    write = sum(w) / nprod * 1024.0
    res = {"kernel": "k_num_heavy_known + k_num_heavy", "scale": scale, "edgefactor": 16,
           "launches": [len(f), len(w)], "products": nprod,
           "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
           "bytes_per_launch": fetch + write, "bytes_per_launch_fetch_doubled": 2 * fetch + write,
           "note": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (KiB x 1024), summed over the heavy kernels per product; "
                   "gfx950 halves FETCH_SIZE for 16-B/lane streams, gathers are uncalibrated"}
    fs = per_dispatch(os.path.join(out, "pmc0"), "k_sym_part").get("FETCH_SIZE", [])
    ws = per_dispatch(os.path.join(out, "pmc1"), "k_sym_part").get("WRITE_SIZE", [])
    if fs and ws:   # the symbolic part kernel over the same runs (one launch per product)
        res["k_sym_part"] = {"launches": [len(fs), len(ws)], "fetch_bytes_per_launch": sum(fs) / nprod * 1024.0,
                             "write_bytes_per_launch": sum(ws) / nprod * 1024.0,
                             "bytes_per_launch": (sum(fs) + sum(ws)) / nprod * 1024.0}
    dst = os.path.join(out, f"{tag}_pmc_heavy.json")   # copied into profiles/ by hand
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps(res))


def all_dispatches(path, counter):
    tot = 0.0
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                tot += float(r["Counter_Value"])
    return tot


def by_kernel(path, counter):
    """counter summed per kernel (short name: the text before the template / argument list)"""
    tot = {}
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("cbg::", "")
                name = name.replace("void ", "").split("(")[0].split("<")[0].strip()
                tot[name] = tot.get(name, 0.0) + float(r["Counter_Value"])
    return tot


def run_product(tag, scale):
    """Whole-product HBM traffic: FETCH_SIZE / WRITE_SIZE summed over EVERY kernel of bench.py runs with 1 and 3
    timed products (+1 warmup, the generator, ...): the difference is two complete products' traffic, so the
    per-product figure carries no generator or set-up kernels -> <tag>_pmc_product.json."""
    out = os.path.join(REPO, "gpurun_out", tag)
    os.makedirs(out, exist_ok=True)
    env = dict(os.environ, TMPDIR="/tmp")
    tot = {}
    for steps in (1, 3):
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(out, f"prod_{ctr}_{steps}")
            cmd = ["timeout", "-s", "KILL", "240", "rocprofv3", "--pmc", ctr, "--output-format", "csv", "-d", d, "-o",
                   "run", "--", sys.executable, os.path.join(REPO, "bench.py"), "--steps", str(steps), "--warmup", "1",
                   "--no-cpu", "--scale", str(scale)]
            r = subprocess.run(cmd, env=env, cwd=REPO, stdout=open(d + ".log", "w"), stderr=subprocess.STDOUT)
            print(f"pass {ctr} steps={steps}: rc={r.returncode}", flush=True)
            if r.returncode != 0:
                sys.exit(r.returncode)
            tot[(ctr, steps)] = all_dispatches(d, ctr) * 1024.0
            tot[(ctr, steps, "k")] = by_kernel(d, ctr)
    fetch = (tot[("FETCH_SIZE", 3)] - tot[("FETCH_SIZE", 1)]) / 2
    write = (tot[("WRITE_SIZE", 3)] - tot[("WRITE_SIZE", 1)]) / 2
    res = {"what": "one whole product (every kernel), R-MAT A*A", "scale": scale, "edgefactor": 16,
           "fetch_bytes_per_product": fetch, "write_bytes_per_product": write,
           "bytes_per_product": fetch + write, "bytes_per_product_fetch_doubled": 2 * fetch + write,
           "note": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (KiB x 1024) summed over all dispatches; (3 products - 1 "
                   "product) / 2; the guide's gfx950 x2 FETCH correction applies to 16-B/lane streams (upper bound)"}
    # per kernel, per product (the same difference): where the product's bytes go
    kern = {}
    for ctr, key in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        a, b = tot[(ctr, 1, "k")], tot[(ctr, 3, "k")]
        for k in set(a) | set(b):
            v = (b.get(k, 0.0) - a.get(k, 0.0)) / 2 * 1024.0
            if abs(v) >= 1e6:
                kern.setdefault(k, {})[key] = v
    res["per_kernel"] = dict(sorted(kern.items(), key=lambda kv: -(kv[1].get("write", 0) + kv[1].get("fetch", 0))))
    dst = os.path.join(out, f"{tag}_pmc_product.json")
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    if len(sys.argv) >= 3 and sys.argv[1] == "run":
        run(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 20)
    elif len(sys.argv) >= 3 and sys.argv[1] == "product":
        run_product(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 20)
    else:
        print(__doc__)
