"""Distributed drivers with the real local kernel: gloo process groups whose ranks all share cuda:0,
each running libcbgpu for its local multiplies and merges (the production path uses RCCL, one GPU per
rank; the schedules are identical).  Checks every rank's output piece exactly."""
import pytest

from dist_support import spawn_case

pytestmark = pytest.mark.gpu

CASES = [(300, 280, 260, 0.03, 0.03, 21), (33, 17, 29, 0.2, 0.15, 5), (5, 64, 6, 0.01, 0.01, 11)]


@pytest.mark.parametrize("world,port", [(2, 29621), (4, 29622), (8, 29623)])
def test_summa_layouts_gloo_gpu(world, port):
    spawn_case(world, "gpu", CASES, port)


MCL_CASES = [(600, 3, 1, (1e-3, 8, 12, 0.9)), (513, 4, 3, (1e-3, 8, 12, 0.9)), (400, 5, 2, (0.05, 5, 9, 0.99))]


@pytest.mark.parametrize("kind", ["gpu", "gpu-rccl-net"])
@pytest.mark.parametrize("world,port", [(2, 29624), (4, 29625), (8, 29626)])
def test_mcl_expansion_gloo_gpu(world, port, kind):
    """Distributed HipMCL expansion (MemEfficientSpGEMM + MCLPruneRecoverySelect) over the host-staged gloo
    transport and over libcbgpu's RCCL grid (every rank its own RCCL node)."""
    from dist_support import run_mcl_case
    spawn_case(world, kind, MCL_CASES, port + (100 if kind != "gpu" else 0), body=run_mcl_case)


INDEX_CASES = [(300, 250, 0.03, 31), (9, 13, 0.3, 23), (3, 4, 0.5, 25)]


@pytest.mark.parametrize("world,port", [(1, 29627), (4, 29628)])
def test_2d_drivers_and_indexing_gloo_gpu(world, port):
    """DoubleBuff / Overlap / Synch and the SpGEMM-based indexing (BoolCopy1st/2nd for Prune,
    PlusTimes for SubsRef_SR / SpAsgn) through libcbgpu, exact against scipy."""
    from dist_support import run_index_case
    spawn_case(world, "gpu", INDEX_CASES, port, body=run_index_case)


FIXTURE_CASES = [("bcsstk01", "pt_f64_hash", "M_matlab")] + \
    [("g500_s10", t, None) for t in ("pt_f64_hash", "pt_i64_hash", "mp_i64_hash", "s2_i64_hash", "sm_i64_hash",
                                     "smb_i64_hash")]


@pytest.mark.parametrize("world,port", [(2, 29631), (4, 29632), (8, 29633)])
def test_reference_fixtures_through_layouts_gloo_gpu(world, port):
    """The reference's golden products (bcsstk01^2 + MATLAB C.mtx as test_mpipspgemm.cpp:101-153 does,
    G500 s10 under PlusTimes f64/i64, MinPlus, Select2nd, SelectMax, SelectMax<bool>) through the
    1x1x2 / 2x2 / 2x2x2 layouts on libcbgpu's native grid (cbg_spgemm_grid), every rank's piece
    checked; Select2nd included (merges follow the inner dimension's order on every layout)."""
    from dist_support import run_fixture_case
    spawn_case(world, "gpu", FIXTURE_CASES, port, body=run_fixture_case)


@pytest.mark.parametrize("world,port", [(4, 29635)])
def test_block_spgemm_and_convert2d_gloo_gpu(world, port):
    """BlockSpGEMM (DoubleBuff block products through libcbgpu) and Convert2D on the G500 s10 fixture."""
    from dist_support import run_block_case
    spawn_case(world, "gpu", [(2, 3), (3, 1)], port, body=run_block_case)


def test_rccl_native_grid_single_rank():
    """libcbgpu's RCCL path (cbg_rccl_unique_id, ncclCommInitRank, ncclCommSplit of row/col/fiber
    communicators) on a one-rank nccl process group: the only RCCL shape one GPU can host (RCCL refuses
    two ranks on one device); the reference fixtures must come out unchanged."""
    from dist_support import run_fixture_case
    spawn_case(1, "gpu-rccl", FIXTURE_CASES[:3], 29634, body=run_fixture_case)


@pytest.mark.parametrize("staged,fiber", [(False, "auto"), (True, "auto"), (False, "reduce")])
@pytest.mark.parametrize("world,port", [(2, 29671), (4, 29672), (8, 29673)])
def test_reference_fixtures_over_rccl_multirank(world, port, staged, fiber, monkeypatch):
    """The production RCCL grid at world 2 / 4 / 8 (1x1x2, 2x2, 2x2x2) with every rank on cuda:0: libcbgpu's
    own communicators (ncclCommInitRank + ncclCommSplit), asynchronous ncclBroadcast of the stage pieces on
    the communication stream, grouped ncclSend/ncclRecv fiber all-to-all-v, ncclAllGather of the sizes.
    Each rank is its own RCCL "node" (NCCL_HOSTID), so RCCL's socket transport carries the bytes.  Panel
    schedule (default) and the staged double-buffered schedule; the reference fixtures (bcsstk01^2 + MATLAB
    C.mtx, G500 s10 under six semirings) must come out on every rank's piece, and RCCL must report the
    grid's group sizes."""
    from dist_support import run_fixture_case
    if world == 4 and fiber == "reduce":
        pytest.skip("one layer: no fiber step")
    if staged:
        monkeypatch.setenv("CBG_GRID_STAGED", "1")
    if fiber == "reduce":   # two layers: the reduction pipeline (codec + merge) instead of the operand gather
        monkeypatch.setenv("CBG_FIBER_GATHER", "0")
    spawn_case(world, "gpu-rccl-net", FIXTURE_CASES, port + (10 if staged else 0) + (20 if fiber == "reduce" else 0),
               body=run_fixture_case)


@pytest.mark.parametrize("world,port", [(2, 29641), (4, 29642), (8, 29643)])
def test_rmat_pieces_built_per_rank_gloo_gpu(world, port):
    """Each rank's A/B pieces built on the device by cbg_rmat_block equal the reference-generated G500
    fixture blocks (s10, s12), and the 1x1x2 / 2x2 / 2x2x2 products of them equal the reference's; at s16
    every layout's pieces equal the same blocks of the one-GPU product (bit-exact: multiplicity values)."""
    from dist_support import run_rmat_case
    spawn_case(world, "gpu", [("g500_s10", 10), ("g500_s12", 12), ("single-gpu", 16)], port, body=run_rmat_case)


@pytest.mark.parametrize("kind", ["gpu", "gpu-rccl-net"])
@pytest.mark.parametrize("world,port", [(2, 29651), (4, 29652), (8, 29653)])
def test_memeff3d_phases_match_reference_gloo_gpu(world, port, kind):
    """MemEfficientSpGEMM3D phasing (ParFriends.h:3214-3705; B pieces per layer chunk, fiber exchange per
    phase, prune per phase): phases 1, 2, 3 reproduce the reference's MemEfficientSpGEMM output
    (golden/mcl.npz) on every rank's piece, with the same branch counts -- over gloo and over RCCL."""
    from dist_support import run_mcl_fixture_case
    spawn_case(world, kind, [1, 2, 3, ("mem", 0.0025)], port + (100 if kind != "gpu" else 0),
               body=run_mcl_fixture_case)


@pytest.mark.parametrize("world,port", [(4, 29661), (8, 29662)])
def test_reference_fixtures_staged_schedule_gloo_gpu(world, port, monkeypatch):
    """The same reference fixtures through the reference's staged SUMMA schedule (CBG_GRID_STAGED=1: q stage
    products + stage merge) -- the default panel schedule must agree with it and with the reference."""
    from dist_support import run_fixture_case
    monkeypatch.setenv("CBG_GRID_STAGED", "1")
    spawn_case(world, "gpu", FIXTURE_CASES, port, body=run_fixture_case)


@pytest.mark.parametrize("kind", ["gpu", "gpu-rccl-net"])
@pytest.mark.parametrize("world,port", [(2, 29681), (4, 29682), (8, 29683)])
def test_galerkin_reference_restriction_multirank_gpu(world, port, kind):
    """BASELINE config 5 distributed: R^T A then (R^T A) R with the reference's R (refrestrict) through libcbgpu's
    grid on the 1x1x2 / 2x2 / 2x2x2 layouts -- over the host-staged gloo transport and over RCCL (every rank its
    own RCCL node) -- every rank's piece of both products equal to the reference's."""
    from dist_support import run_galerkin_case
    spawn_case(world, kind, ["SUMMA3D", "multiply"], port + (10 if kind != "gpu" else 0), body=run_galerkin_case)


@pytest.mark.parametrize("kind,port", [("gpu", 29691), ("gpu-rccl-net", 29692)])
def test_fiber_row_gaps_tall_sparse(kind, port):
    """1x1x2 fiber exchange of tall, very sparse products through the 16-bit row gaps (k_gap_encode /
    k_gap_decode): first rows above 65534 and gaps above it (escapes, also mid-column), columns of one 64-entry
    chunk and of hundreds; integer values (u16 on the wire), compared exactly with scipy's product."""
    spawn_case(2, kind, [(2000000, 3000, 96, 5e-6, 0.002, 5),
                         (1000000, 3000, 120, 2e-5, 0.002, 7),
                         (300000, 500, 64, 1e-3, 0.2, 9)], port)


# (n, k, m, density A, density B, seed, value kind, bound on wire bytes per output entry or None)
FIBER_CASES = [(4000, 600, 300, 0.05, 0.05, 41, "small", 3.0),        # dense runs: 1-byte gaps and values
               (300000, 500, 64, 1e-3, 0.2, 43, "small", None),       # gaps around 2^8..2^14
               (2000000, 3000, 96, 5e-6, 0.002, 45, "wide", None),    # gaps above 2^16 (u16 escapes / 3-byte varint)
               (3000, 400, 200, 0.05, 0.05, 47, "huge", None),        # products above 2^32: f64 values
               (3000, 400, 200, 0.05, 0.05, 49, "real", None),        # reals: f64
               (50, 40, 30, 0.0, 0.0, 51, "small", None)]             # empty product


@pytest.mark.parametrize("env", ["default", "CBG_FIBER_VARINT=0", "CBG_FIBER_GAPS=0"])
@pytest.mark.parametrize("kind,port", [("gpu", 29701), ("gpu-rccl-net", 29711)])
def test_fiber_wire_formats(kind, port, env, monkeypatch):
    """The fiber pipeline's per-message wire formats (varint / 16-bit-gap / int32 rows; varint / u16 / f32 / f64
    values) at world 2 over gloo and over RCCL, exact against scipy, with the varint codes on and off."""
    from dist_support import run_fiber_case
    off = {"default": 0, "CBG_FIBER_VARINT=0": 1, "CBG_FIBER_GAPS=0": 2}[env]
    if env != "default":
        k, v = env.split("=")
        monkeypatch.setenv(k, v)
    cases = FIBER_CASES if env == "default" else [c[:-1] + (None,) for c in FIBER_CASES]
    spawn_case(2, kind, cases, port + off, body=run_fiber_case)


@pytest.mark.parametrize("fiber", ["auto", "reduce"])
@pytest.mark.parametrize("world,port", [(2, 29681), (8, 29683)])
def test_fiber_gather_and_reduction_on_rmat(world, port, fiber, monkeypatch):
    """Two-layer grids (1x1x2, 2x2x2) over libcbgpu's RCCL grid on an R-MAT s14 A*A: the grid takes the fiber gather of
    the layer operands (operands on the fiber, no merge) unless CBG_FIBER_GATHER=0 forces the reduction of partial
    products; either way every rank's piece equals the same block of the one-GPU product (multiplicities: bit-exact)."""
    from dist_support import run_rmat_case
    if fiber == "reduce":
        monkeypatch.setenv("CBG_FIBER_GATHER", "0")
    spawn_case(world, "gpu-rccl-net", [("fiber-mode", 14)], port + (1 if fiber == "reduce" else 0), body=run_rmat_case)
