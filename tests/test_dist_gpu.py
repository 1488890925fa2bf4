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


@pytest.mark.parametrize("world,port", [(2, 29624), (4, 29625), (8, 29626)])
def test_mcl_expansion_gloo_gpu(world, port):
    from dist_support import run_mcl_case
    spawn_case(world, "gpu", MCL_CASES, port, body=run_mcl_case)


INDEX_CASES = [(300, 250, 0.03, 31), (9, 13, 0.3, 23), (3, 4, 0.5, 25)]


@pytest.mark.parametrize("world,port", [(1, 29627), (4, 29628)])
def test_2d_drivers_and_indexing_gloo_gpu(world, port):
    """DoubleBuff / Overlap / Synch and the SpGEMM-based indexing (BoolCopy1st/2nd for Prune,
    PlusTimes for SubsRef_SR / SpAsgn) through libcbgpu, exact against scipy."""
    from dist_support import run_index_case
    spawn_case(world, "gpu", INDEX_CASES, port, body=run_index_case)
