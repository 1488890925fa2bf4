"""Diagnostic: per-phase cycle breakdown of k_num_heavy_known from the stamps build (tools/diag/libcbgpu.so), on the
s20 A*A and on a rank-share-like product at scale 22 (A(0:2^21, 0:2^21) * A(0:2^21, 0:2^20): 2^21 rows, half the
column density of the s20 product).  usage: python tools/diag_known.py"""
import ctypes
import os
import sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from combblas_amd import _abi  # noqa: E402
_abi.LIB_PATH = os.path.join(HERE, "diag", "libcbgpu.so")
import combblas_amd as cb  # noqa: E402

lib = _abi.lib()
lib.cbg_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
ctx = cb.Context(0)
PT = cb.PlusTimesSRing("f64")
names = {1: "loop top", 6: "a: clear values, rows out, directory", 7: "a: barrier", 8: "b: bits",
         9: "b: next unit's rows issued", 2: "b: barrier", 3: "stage chunk (fetch + scan + barrier)",
         4: "expand chunk (search, gathers, slots, acc, barrier)", 10: "d: values out", 5: "d: ring + barrier"}


def run(label, A, B):
    C = cb.LocalSpGEMMHash(PT, A, B)
    C.free()
    buf = (ctypes.c_uint64 * 32)()
    lib.cbg_debug_stamps(buf, 1)
    C = cb.LocalSpGEMMHash(PT, A, B)
    p = ctx.last_profile()
    C.free()
    lib.cbg_debug_stamps(buf, 0)
    s = list(buf)
    tot = sum(s[i] for i in names)
    print(f"== {label}: heavy {p['heavy_ms']:.2f} ms, known units {p['known_items']}, heavy multiplies "
          f"{p['heavy_multiplies']}, outputs {p['heavy_nnz_c']}, B nonzeros {p['heavy_nnz_b']}")
    for i, nm in names.items():
        print(f"  phase {i} {nm:55s} {s[i]:16d} cycles  {100.0 * s[i] / max(tot, 1):5.1f}%")
    if p["known_items"]:
        print(f"  per unit: {tot / p['known_items'] / 1e3:.1f} k cycles (summed over workgroups' thread 0)")


A = ctx.generate_rmat(20, 16)
run("s20 A*A", A, A)
A.free()
n = 1 << 22
Ar = ctx.rmat_block(22, 0, n // 2, 0, n // 2)
Bc = ctx.rmat_block(22, 0, n // 2, 0, n // 4)
run("s22 A(0:2^21,0:2^21)*A(0:2^21,0:2^20)", Ar, Bc)
