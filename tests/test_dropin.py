"""The C++ drop-in header (include/combblas_gpu.h) against the reference's own types and kernels.

tests/dropin/dropin_test.cpp is compiled against the reference headers (build container only, by
__graft_entry__.build() or here) and links libcbgpu.so; on a GPU it compares gpu::LocalSpGEMMHash,
gpu::MultiwayMerge and gpu::EstimateLocalFLOP with the reference's LocalSpGEMMHash / MultiwayMerge /
EstimateLocalFLOP in one process, plus a semiring without a device functor (reference CPU template),
and the distributed drivers (gpu::Mult_AnXBn_Synch etc.) against the reference's Mult_AnXBn_Synch."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
BIN = os.path.join(HERE, "dropin", "_bin", "dropin_test")


def _build():
    if os.path.isdir("/root/reference") and os.path.exists("/opt/conda/include/mpi.h"):
        subprocess.run(["make", "-C", os.path.join(HERE, "dropin")], check=True, capture_output=True)
    return os.path.exists(BIN)


def test_dropin_builds_and_reports_missing_device():
    """CPU container: the header compiles against the reference and the device path fails loudly."""
    if not _build():
        pytest.skip("reference headers not available (GPU box): covered by the gpu test")
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is visible: the gpu tests cover the device path")
    r = subprocess.run([BIN, "--expect-no-gpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "device path:" in r.stdout


@pytest.mark.gpu
def test_dropin_matches_reference_on_gpu():
    if not os.path.exists(BIN):
        pytest.skip("dropin_test not built (needs the reference headers in the build container)")
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=150)
    assert r.returncode == 0 and "DROPIN OK" in r.stdout, r.stdout + r.stderr


MPIRUN = "/opt/conda/bin/mpirun"


def mpi_cmd(world, args, transport):
    """mpirun line for `world` ranks of dropin_test sharing cuda:0.  transport "rccl" (the drop-in's default: the
    library's RCCL communicators) gives every rank its own NCCL_HOSTID through MPICH's MPMD syntax, so each rank is its
    own RCCL "node" and RCCL's socket transport carries the bytes (RCCL refuses two ranks of one host on one device);
    "mpi" selects the host-staged MPI transport (CBG_GRID_TRANSPORT=mpi)."""
    cmd = [MPIRUN]
    if transport == "mpi":
        return cmd + ["-genv", "CBG_GRID_TRANSPORT", "mpi", "-np", str(world), BIN] + list(args)
    cmd += ["-genv", "NCCL_SOCKET_IFNAME", "lo", "-genv", "NCCL_IB_DISABLE", "1"]
    for r in range(world):
        if r:
            cmd.append(":")
        cmd += ["-np", "1", "-env", "NCCL_HOSTID", f"cbg-dropin-{r}", BIN] + list(args)
    return cmd


def assert_grid(out, world, q, L, transport):
    """Every rank reports the grid its distributed drivers ran over (cbg_grid_query): RCCL's own member counts of
    the world / row / column / fiber communicators, or the MPI transport's group sizes."""
    want = f"GRID rccl={1 if transport == 'rccl' else 0} world={world} row={q} col={q} fiber={L}"
    assert out.count(want) == world, (want, out)


@pytest.mark.gpu
@pytest.mark.parametrize("transport", ["rccl", "mpi"])
def test_dropin_distributed_drivers_4_ranks_on_gpu(transport):
    """gpu::Mult_AnXBn_Synch / DoubleBuff / Overlap / PSpGEMM at 4 MPI ranks (2x2 CommGrid, ranks sharing
    cuda:0; libcbgpu's grid over its own RCCL communicators, or over the SpParMat's MPI communicators) against the
    reference's own Mult_AnXBn_Synch on the same operands, block by block (the reference's duplicates summed); and
    gpu::MCLPruneRecoverySelect on the 2x2 grid (columns gathered along the processor column, pruned on the device)
    against the reference's MCLPruneRecoverySelect (ParFriends.h:185-353) on the same SpParMat."""
    if not os.path.exists(BIN) or not os.path.exists(MPIRUN):
        pytest.skip("dropin_test or MPICH's mpirun not available")
    r = subprocess.run(mpi_cmd(4, [], transport), capture_output=True, text=True, timeout=150)
    assert r.returncode == 0 and r.stdout.count("DROPIN OK") == 4, r.stdout + r.stderr
    # ten more Mult_AnXBn_Synch calls on the same CommGrid set up no communicator (the grid is cached)
    reps = [line for line in r.stdout.splitlines() if line.startswith("REPEAT")]
    import re
    setups = [re.search(r"setups_before=(\d+) setups_after=(\d+)", x).groups() for x in reps]
    assert len(reps) == 4 and all(b == a for b, a in setups), reps
    print("\n".join(reps))
    assert_grid(r.stdout, 4, 2, 1, transport)


def _write_mtx(path, nrow, ncol, cp, ir, val):
    """MatrixMarket coordinate real general, 1-based (what ParallelReadMM reads, onebased = true)."""
    import numpy as np
    cols = np.repeat(np.arange(ncol), np.diff(cp))
    with open(path, "w") as f:
        f.write("%%MatrixMarket matrix coordinate real general\n")
        f.write(f"{nrow} {ncol} {len(ir)}\n")
        for r, c, v in zip(ir, cols, val):
            f.write(f"{int(r) + 1} {int(c) + 1} {float(v)!r}\n")


def _fixture_mtx(tmp_path):
    """bcsstk01 (A) and MATLAB's bcsstk01^2 (3DSpGEMM/matlab/C.mtx, held in bcsstk01.npz), and the reference's
    Graph500 s10 matrix (integer multiplicities), written from the committed fixtures."""
    import numpy as np
    z = np.load(os.path.join(HERE, "golden", "bcsstk01.npz"))
    n = int(z["A_shape"][0])
    fa, fc, fg = (str(tmp_path / x) for x in ("A.mtx", "C.mtx", "G.mtx"))
    _write_mtx(fa, n, n, z["A_cp"], z["A_ir"], z["A_val"])
    _write_mtx(fc, n, n, z["M_matlab_cp"], z["M_matlab_ir"], z["M_matlab_val"])
    g = np.load(os.path.join(HERE, "golden", "g500_s10.npz"))
    m = int(g["A_shape"][0])
    _write_mtx(fg, m, m, g["A_cp"], g["A_ir"], g["A_val"])
    return fa, fc, fg


@pytest.mark.gpu
@pytest.mark.parametrize("transport", ["rccl", "mpi"])
@pytest.mark.parametrize("q,L", [(1, 2), (2, 1), (1, 4), (2, 2)])
def test_dropin_3dspgemm_and_summa3d_on_gpu(q, L, transport, tmp_path):
    """gpu::multiply / gpu::SUMMALayer (3DSpGEMM/Multiplier.h:10-61, SUMMALayer.h:24-97) on a CCGrid of
    q x q x L MPI ranks sharing cuda:0, set up as test_mpipspgemm.cpp:101-153 does (ReadMat + SplitMat of
    bcsstk01), against the reference's multiply / SUMMALayer on the same split pieces and against MATLAB's
    C.mtx; and gpu::Mult_AnXBn_SUMMA3D against the reference's Mult_AnXBn_SUMMA3D on SpParMat3D operands
    with L layers (bcsstk01 within 1e-12 of sum|a*b|, Graph500 s10 bit-exact), every rank's piece, where the
    world is a square (the reference's SpParMat3D is built from a 2D SpParMat on a square CommGrid: 2x2x1 and
    1x1x4 here; 1x1x2 and 2x2x2 exercise the split-3D driver)."""
    if not os.path.exists(BIN) or not os.path.exists(MPIRUN):
        pytest.skip("dropin_test or MPICH's mpirun not available")
    fa, fc, fg = _fixture_mtx(tmp_path)
    world = q * q * L
    r = subprocess.run(mpi_cmd(world, ["--3d", str(q), str(L), fa, fc, fg], transport), capture_output=True,
                       text=True, timeout=150)
    assert r.returncode == 0 and r.stdout.count("DROPIN3D OK") == world, r.stdout + r.stderr
    assert_grid(r.stdout, world, q, L, transport)


@pytest.mark.gpu
@pytest.mark.parametrize("q", [1, 2])
@pytest.mark.parametrize("name", ["poisson12", "g500_s10"])
def test_dropin_restriction_op_on_gpu(q, name, tmp_path):
    """gpu::RestrictionOp (3DSpGEMM/RestrictionOp.h:196-291) on a CCGrid layer of q x q MPI ranks: the layer's pieces
    go to the device on the layer's rank 0, and every rank's R and R^T blocks (SpParMat distribution of the layer
    grid) must hold the reference's one-rank R -- oracle/_ref/refrestrict's output in golden/restriction.npz."""
    if not os.path.exists(BIN) or not os.path.exists(MPIRUN):
        pytest.skip("dropin_test or MPICH's mpirun not available")
    import numpy as np
    z = np.load(os.path.join(HERE, "golden", "restriction.npz"))
    if name.startswith("poisson"):
        import sys
        sys.path.insert(0, os.path.dirname(HERE))
        from combblas_amd.inputs import poisson3d
        n, cp, ir, val = poisson3d(int(name[len("poisson"):]))
    else:
        cp, ir = z[f"{name}_cp"], z[f"{name}_ir"]
        n = len(z[f"{name}_agg"])
        val = np.ones(len(ir))
    fa, fg = str(tmp_path / "A.mtx"), str(tmp_path / "agg.txt")
    _write_mtx(fa, n, n, cp, ir, val)
    np.savetxt(fg, z[f"{name}_agg"].astype(np.int64), fmt="%d")
    r = subprocess.run(mpi_cmd(q * q, ["--restrict", str(q), fa, fg], "rccl"), capture_output=True, text=True,
                       timeout=150)
    assert r.returncode == 0 and r.stdout.count("DROPINR OK") == q * q, r.stdout + r.stderr
