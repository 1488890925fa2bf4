"""CPU-only checks of the C ABI library: it loads without a GPU, exports exactly what include/cbgpu.h
declares, and its host-side pieces (status strings, generator) work without a device."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from helpers import REPO

HEADER = os.path.join(REPO, "include", "cbgpu.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(cbg_[a-z0-9_]+)\s*\(", src)))


def test_library_loads_and_exports_every_declared_symbol():
    from combblas_amd import _abi
    lib = _abi.lib()
    names = declared_functions()
    assert len(names) >= 15
    out = subprocess.run(["nm", "-D", "--defined-only", _abi.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (cbg_\w+)", out))
    missing = [n for n in names if n not in exported]
    assert not missing, f"declared in cbgpu.h but not exported: {missing}"
    for n in names:
        assert hasattr(lib, n)
    # the python binding declares every entry point with a signature
    assert set(names) == set(_abi.SIGNATURES), set(names) ^ set(_abi.SIGNATURES)


def test_no_oracle_in_product_library():
    """The product library must not link or contain the oracle (no CPU fallback path)."""
    from combblas_amd import _abi
    out = subprocess.run(["nm", "-D", _abi.LIB_PATH], capture_output=True, text=True).stdout
    assert "orc_" not in out
    ldd = subprocess.run(["ldd", _abi.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in ldd


def test_abi_version_and_strerror():
    from combblas_amd import _abi
    lib = _abi.lib()
    assert lib.cbg_abi_version() == 4
    assert b"3002" in lib.cbg_strerror(3002)
    assert b"BoolCopy" in lib.cbg_strerror(13)


def test_struct_layouts_match_header(tmp_path):
    """Every ctypes mirror has the C compiler's size and field offsets of include/cbgpu.h's struct."""
    import shutil
    import subprocess
    from combblas_amd import _abi
    structs = {"cbg_dcsc_view": _abi.DcscView, "cbg_csc_result": _abi.CscResult, "cbg_profile": _abi.Profile,
               "cbg_mcl_stats": _abi.MclStats, "cbg_grid_stats": _abi.GridStats, "cbg_codec_stats": _abi.CodecStats,
               "cbg_grid_info": _abi.GridInfo, "cbg_transport": _abi.Transport, "cbg_host_csc": _abi.HostCsc}
    assert ctypes.sizeof(_abi.DcscView) == 80 and ctypes.sizeof(_abi.CscResult) == 72
    if shutil.which("gcc") is None:
        pytest.skip("no C compiler")
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "cbgpu.h"', "int main(void) {"]
    for cname, py in structs.items():
        lines.append(f'  printf("{cname} size %zu\\n", sizeof({cname}));')
        for f in py._fields_:
            lines.append(f'  printf("{cname} {f[0]} %zu\\n", offsetof({cname}, {f[0]}));')
    lines.append("  return 0;\n}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)], check=True)
    got = {}
    for line in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.splitlines():
        c, f, v = line.split()
        got[(c, f)] = int(v)
    for cname, py in structs.items():
        assert got[(cname, "size")] == ctypes.sizeof(py), cname
        for f in py._fields_:
            assert got[(cname, f[0])] == getattr(py, f[0]).offset, (cname, f[0])


def test_init_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    import combblas_amd as cb
    with pytest.raises(cb.CbgError) as ei:
        cb.Context(0)
    assert ei.value.status == 12


def test_rmat_generator_properties():
    import combblas_amd as cb
    n, cp, ir, val = cb.generate_rmat_host(12, 16, seed=3)
    assert n == 4096 and len(cp) == n + 1 and cp[0] == 0
    assert val.sum() == 16 * 4096                          # multiplicities add up to all edges
    assert np.all(np.diff(cp) >= 0)
    for j in range(0, n, 97):
        seg = ir[cp[j]:cp[j + 1]]
        assert np.all(np.diff(seg) > 0)                    # rows sorted, duplicates merged
    n2, cp2, ir2, val2 = cb.generate_rmat_host(12, 16, seed=3)
    assert np.array_equal(cp, cp2) and np.array_equal(ir, ir2) and np.array_equal(val, val2)
    n3, cp3, _, _ = cb.generate_rmat_host(12, 16, seed=4)
    assert not np.array_equal(cp, cp3)


def kron_cases():
    import json
    return json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "kron.json")))["cases"]


@pytest.mark.parametrize("case", [c for c in kron_cases() if c["scale"] <= 18],
                         ids=lambda c: f"s{c['scale']}_seed{c['seed']}")
def test_rmat_host_matches_reference_generator(case):
    """cbg_rmat_host reproduces the reference's GenGraph500Data(packed) + SpParMat(DEL) matrix exactly:
    canonical SHA-256 of refprobe `gen` output (tests/golden/make_golden_kron.py, kron.json)."""
    import combblas_amd as cb
    from helpers import canonical_sha256
    n, cp, ir, val = cb.generate_rmat_host(case["scale"], case["edgefactor"], seed=case["seed"])
    assert len(ir) == case["nnz"] and val.sum() == case["sum_val"]
    assert canonical_sha256(cp, ir, val) == case["sha256"]


def test_rmat_host_equals_reference_fixture_arrays():
    """The whole s10 / s12 reference matrices stored in the fixtures, array by array."""
    import combblas_amd as cb
    from helpers import load_fixture
    for scale in (10, 12):
        z = load_fixture(f"g500_s{scale}")
        n, cp, ir, val = cb.generate_rmat_host(scale, 16)
        assert np.array_equal(cp, z["A_cp"]) and np.array_equal(ir, z["A_ir"]) and np.array_equal(val, z["A_val"])


def test_loader_refuses_another_abi_version(monkeypatch):
    """The library writes structs the caller allocates (cbg_profile, cbg_grid_stats): _abi.lib() refuses a library whose
    cbg_abi_version() is not the one these bindings were written for."""
    from combblas_amd import _abi
    saved = _abi._lib
    try:
        monkeypatch.setattr(_abi, "_lib", None)
        monkeypatch.setattr(_abi, "ABI_VERSION", _abi.ABI_VERSION + 1)
        with pytest.raises(OSError, match="cbg_abi_version"):
            _abi.lib()
    finally:
        _abi._lib = saved
