#!/usr/bin/env python3
"""Benchmark tuning variants (tools/var/<name>/libcbgpu.so, `make -C combblas_amd/csrc var`) with the
same bench.py code path.  usage: python tools/var_bench.py name [name ...] -- [bench args]
Each variant runs in its own child process (one library per process)."""
import os
import runpy
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)

if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--one":
        sys.path.insert(0, REPO)
        from combblas_amd import _abi
        if sys.argv[2] != "main":   # "main": the in-tree product library
            _abi.LIB_PATH = os.path.join(HERE, "var", sys.argv[2], "libcbgpu.so")
        sys.argv = [os.path.join(REPO, "bench.py")] + sys.argv[3:]
        runpy.run_path(sys.argv[0], run_name="__main__")
        sys.exit(0)
    args = sys.argv[1:]
    names, rest = (args[:args.index("--")], args[args.index("--") + 1:]) if "--" in args else (args, [])
    for n in names:
        r = subprocess.run([sys.executable, __file__, "--one", n] + rest, capture_output=True, text=True,
                           timeout=600)
        line = (r.stdout.strip().splitlines() or [""])[-1]
        if r.returncode == 0:
            import json
            j = json.loads(line)
            if "ms_per_step" in j:
                print(n, "ms/step %.2f" % j["ms_per_step"], "nnz_C", j["config"].get("nnz_C"), j.get("phases_ms"),
                      flush=True)
            else:   # bench.py --rank-share: one line per rank
                for x in r.stdout.strip().splitlines():
                    if x.startswith("{"):
                        d = json.loads(x)
                        print(n, "rank", d.get("rank"), {k: d.get(k) for k in ("local_ms", "symbolic_ms", "heavy_ms",
                                                                              "merge_ms", "heavy_GBps")}, flush=True)
        else:
            print(n, "rc", r.returncode, r.stderr[-2000:], flush=True)
        if r.returncode != 0:
            sys.exit(r.returncode)
