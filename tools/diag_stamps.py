"""Diagnostic: per-phase cycle breakdown of k_num_heavy from the stamps build (tools/diag/libcbgpu.so).
usage: python tools/diag_stamps.py [scale]"""
import ctypes, os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from combblas_amd import _abi
_abi.LIB_PATH = os.path.join(HERE, "diag", "libcbgpu.so")
import combblas_amd as cb
import numpy as np
scale = int(sys.argv[1]) if len(sys.argv) > 1 else 20
lib = _abi.lib()
lib.cbg_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = (ctypes.c_uint64 * 32)()
ctx = cb.Context(0)
n, cp, ir, val = cb.generate_rmat_host(scale, 16, seed=1)
A = cb.SpDCCols.from_csc(ctx, n, n, cp, ir, val)
C = cb.LocalSpGEMMHash(cb.PlusTimesSRing("f64"), A, A); C.free()
lib.cbg_debug_stamps(buf, 1)
C = cb.LocalSpGEMMHash(cb.PlusTimesSRing("f64"), A, A)
prof = ctx.last_profile(); C.free()
lib.cbg_debug_stamps(buf, 0)
s = list(buf)
names = {0: "item setup", 1: "(unused)", 2: "table init", 3: "stage (fetch+scan)",
         4: "expand", 5: "compaction end (dense path / final sync)", 6: "post-expand sync", 7: "hash count+scan",
         8: "hash compact_runs+stores"}
tot = sum(s[i] for i in range(9))
for i in range(9):
    print(f"phase {i} {names[i]:40s} {s[i]:16d} cycles  {100.0*s[i]/max(tot,1):5.1f}%")
for i, nm in ((15, "  home count atomics+sync"), (16, "  scan+rewrite+sync"), (17, "  positions+sync"),
              (18, "  staging writes+sync"), (19, "  group sort+sync"), (20, "  coalesced copy (thread 0)")):
    print(f"phase {i} {nm:40s} {s[i]:16d} cycles")
print("runs", s[19], "keys in runs", s[20], "max run", s[21], "sum L^2", s[22])
print(f"rank single-chunk: sweep 1 (rows + marks) {s[24]} cycles, directory {s[25]} cycles "
      f"(phase 4 'expand' = sweep 2 for those units)")
print("k_sym_part: clear", s[26], "expand", s[27], "count+scan", s[28], "rows+subwindow counts", s[29])
if s[30]:
    print("k_sym_part per item (cycles): items", s[30], "clear %.0f expand %.0f count+scan %.0f rows %.0f" %
          tuple(s[i] / s[30] for i in (26, 27, 28, 29)))
print("units", s[10], "chunks", s[11], "multiplies", s[12], "hash units", s[13])
print("profile", {k: prof[k] for k in ("numeric_ms", "symbolic_ms", "total_ms")})
