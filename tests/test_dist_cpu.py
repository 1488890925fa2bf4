"""Distributed drivers on CPU: gloo process groups with a scipy local multiply (TEST INFRASTRUCTURE).

Checks the mandated layouts end to end: 1x1x2 (2 ranks: fiber exchange, no broadcast),
2x2 SUMMA (4 ranks: row/column broadcasts, 2 stages, merge), 2x2x2 (8 ranks: both), on square and
rectangular products with empty blocks; every rank checks its output piece exactly against the global
product and the multiplies add up to estimateFLOP of the whole product.
"""
import pytest

from dist_support import spawn_case

CASES = [(60, 50, 40, 0.08, 0.1, 3), (33, 17, 29, 0.2, 0.15, 5), (7, 5, 9, 0.3, 0.3, 9), (5, 64, 6, 0.01, 0.01, 11)]


@pytest.mark.parametrize("world,port", [(2, 29611), (4, 29612), (8, 29613)])
def test_summa_layouts_gloo_cpu(world, port):
    spawn_case(world, "scipy", CASES, port)


MCL_CASES = [(300, 3, 1, (1e-3, 8, 12, 0.9)), (257, 4, 3, (1e-3, 8, 12, 0.9)), (200, 5, 2, (0.05, 5, 9, 0.99))]


@pytest.mark.parametrize("world,port", [(2, 29614), (4, 29615), (8, 29616)])
def test_mcl_expansion_gloo_cpu(world, port):
    from dist_support import run_mcl_case
    spawn_case(world, "scipy", MCL_CASES, port, body=run_mcl_case)


INDEX_CASES = [(40, 30, 0.1, 21), (9, 13, 0.3, 23), (3, 4, 0.5, 25)]


@pytest.mark.parametrize("world,port", [(1, 29617), (4, 29618)])
def test_2d_drivers_and_indexing_gloo_cpu(world, port):
    """Mult_AnXBn_Synch / DoubleBuff / Overlap and SubsRef_SR / Prune / PruneFull / SpAsgn on 1x1 and
    2x2 grids (SpParMat.cpp:2028-2562, ParFriends.h:799-1235) against scipy on the global matrices."""
    from dist_support import run_index_case
    spawn_case(world, "scipy", INDEX_CASES, port, body=run_index_case)


BLOCK_CASES = [(2, 3), (3, 1), (1, 1)]


@pytest.mark.parametrize("world,port", [(1, 29619), (4, 29620)])
def test_block_spgemm_and_convert2d_gloo_cpu(world, port):
    """BlockSpGEMM / BlockSplit and SpParMat3D::Convert2D on the reference's G500 s10 fixture product."""
    from dist_support import run_block_case
    spawn_case(world, "scipy", BLOCK_CASES, port, body=run_block_case)


@pytest.mark.parametrize("world,port", [(2, 29641), (4, 29642)])
def test_rmat_pieces_built_per_rank_gloo_cpu(world, port):
    """SpParMat3D.from_rmat: each rank builds only its own A/B pieces of the reference's Graph500 matrix;
    pieces equal the reference-generated s10 fixture blocks and the SUMMA3D product equals its product."""
    from dist_support import run_rmat_case
    spawn_case(world, "scipy", [("g500_s10", 10)], port, body=run_rmat_case)


@pytest.mark.parametrize("world,port", [(2, 29651), (8, 29652)])
def test_memeff3d_phases_match_reference_gloo_cpu(world, port):
    """MemEfficientSpGEMM3D phasing (ParFriends.h:3214-3705; B pieces per layer chunk, fiber exchange per
    phase, prune per phase): phases 1, 2, 3 reproduce the reference's MemEfficientSpGEMM output
    (golden/mcl.npz) on every rank's piece, with the same branch counts."""
    from dist_support import run_mcl_fixture_case
    spawn_case(world, "scipy", [1, 2, 3, ("mem", 0.0025)], port, body=run_mcl_fixture_case)


@pytest.mark.parametrize("world,port", [(2, 29661), (4, 29662), (8, 29663)])
def test_galerkin_reference_restriction_gloo_cpu(world, port):
    """R^T A then (R^T A) R with the reference's R on the 1x1x2 / 2x2 / 2x2x2 layouts (SUMMA3D and multiply)."""
    from dist_support import run_galerkin_case
    spawn_case(world, "scipy", ["SUMMA3D", "multiply"], port, body=run_galerkin_case)
