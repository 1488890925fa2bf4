"""The restriction-operator oracle (oracle/restriction.py) against the reference's own RestrictionOp output
(tests/golden/restriction.npz, made by oracle/_ref/refrestrict; see make_golden_restriction.py)."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
from helpers import load_fixture  # noqa: E402
from restriction import MT19937, restriction_op, std_shuffle_minstd  # noqa: E402
from combblas_amd.inputs import poisson3d  # noqa: E402

CASES = ["poisson6", "poisson12", "poisson80", "g500_s10", "unsym700"]


def case_input(z, name):
    if name.startswith("poisson"):
        n, cp, ir, _ = poisson3d(int(name[len("poisson"):]))
        return n, cp, ir
    return len(z[f"{name}_agg"]), z[f"{name}_cp"], z[f"{name}_ir"].astype(np.int64)


@pytest.mark.parametrize("name", CASES)
def test_oracle_restriction_matches_reference(name):
    """Same MIS-2 set, same parents, same column permutation: R equals the reference's entry for entry."""
    z = load_fixture("restriction")
    n, cp, ir = case_input(z, name)
    nagg, rcp, rir, rval, st = restriction_op(n, cp, ir)
    assert nagg == int(z[f"{name}_nagg"])
    agg = np.empty(n, np.int64)
    for c in range(nagg):
        agg[rir[rcp[c]:rcp[c + 1]]] = c
    assert np.array_equal(agg, z[f"{name}_agg"])
    assert np.all(rval == 1.0)


def test_mt19937_known_answer():
    """MTRand(5489) = the MT19937 reference sequence (10000th output 4123659995)."""
    mt = MT19937(5489)
    s = mt.randint(10000)
    assert int(s[0]) == 3499211612 and int(s[-1]) == 4123659995


def test_shuffle_is_a_permutation_both_branches():
    for n in (1, 2, 3, 10, 46340, 46341):
        p = std_shuffle_minstd(n, 1383098845)
        assert np.array_equal(np.sort(p), np.arange(n))
