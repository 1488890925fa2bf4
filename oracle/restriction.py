"""oracle/restriction.py -- CPU restatement of the reference's Galerkin restriction operator.

TEST INFRASTRUCTURE ONLY.  This is a parity checker: only tests/ may import it.  The product path
(libcbgpu.so, cbg_restriction_op) never loads, calls or falls back to it.

Pinned against the reference itself: oracle/_ref/refrestrict runs the reference's RestrictionOp at one
rank under its DETERMINISTIC switch, and tests/golden/restriction.npz holds its R for 3D Poisson grids
(tests/golden/make_golden_restriction.py); tests/test_oracle_restriction.py checks this restatement
against every one of them.

Algorithm restated (file:line refer to /root/reference):
  MTRand(1)                   psort-1.0/include/psort/MersenneTwister.h:137-147, 179-196, 283-314
                              (MT19937, init_genrand seeding, rand() = randInt() / 4294967295.0);
                              RestrictionOp.h:15-16 seeds the global generator with 1 (DETERMINISTIC)
  MIS2                        3DSpGEMM/RestrictionOp.h:116-193 -- every round draws one value per
                              candidate in ascending vertex order, takes the minimum over the 1- and 2-hop
                              candidate neighbourhoods (SpMV with Select2ndMinSR, :146-152), admits the
                              candidates whose value is <= that minimum (:158-161), and removes them and
                              their 1- and 2-hop neighbours from the candidates (:164-183)
  RestrictionOp               3DSpGEMM/RestrictionOp.h:196-291 -- B = pattern(A) without loops, B += B^T;
                              parent = the MIS-2 neighbour (MIS2verifySR, :216-222) or the vertex itself;
                              one draw per parented vertex in ascending order (:225-229); an unparented
                              vertex takes the parent of its neighbour with the smallest draw
                              (Select2ndRandSR, :63-84; on equal draws the later neighbour in column order,
                              the SPA accumulation order of SpImpl.cpp:233-256); R(i, c) = 1 where column c
                              is the parent's rank among the MIS-2 vertices (:256-262), then the columns
                              are permuted by RandPerm (:268-275)
  FullyDistVec::RandPerm      include/CombBLAS/FullyDistVec.cpp:783-900 at one rank: std::shuffle of
                              0..nagg-1 with std::default_random_engine(1383098845) (libstdc++ 11:
                              bits/stl_algo.h shuffle, bits/uniform_int_dist.h downscaling, minstd_rand0)
The reference is only deterministic with one OpenMP thread: FullyDistSpVec::Apply draws from the shared
generator inside an OpenMP loop (FullyDistSpVec.h:237-246), so the fixtures are generated serially.
"""
import numpy as np

_UP, _LO, _MATA = np.uint32(0x80000000), np.uint32(0x7FFFFFFF), np.uint32(0x9908B0DF)


class MT19937:
    """MersenneTwister.h's MTRand: uint32 stream (randInt) of a one-word seed."""

    def __init__(self, seed):
        mt = np.zeros(624, np.uint64)
        mt[0] = seed & 0xFFFFFFFF
        for i in range(1, 624):
            p = int(mt[i - 1])
            mt[i] = (1812433253 * (p ^ (p >> 30)) + i) & 0xFFFFFFFF
        self.mt = mt.astype(np.uint32)
        self.idx = 624

    def _twist(self):
        mt = self.mt

        def tw(m, s0, s1):
            y = (s0 & _UP) | (s1 & _LO)
            return m ^ (y >> np.uint32(1)) ^ ((s1 & np.uint32(1)) * _MATA)
        mt[0:227] = tw(mt[397:624], mt[0:227], mt[1:228])
        mt[227:454] = tw(mt[0:227], mt[227:454], mt[228:455])
        mt[454:623] = tw(mt[227:396], mt[454:623], mt[455:624])
        mt[623] = tw(mt[396:397], mt[623:624], mt[0:1])[0]
        self.idx = 0

    def randint(self, k):
        out = np.empty(k, np.uint32)
        o = 0
        while o < k:
            if self.idx == 624:
                self._twist()
            t = min(624 - self.idx, k - o)
            y = self.mt[self.idx:self.idx + t].copy()
            y ^= y >> np.uint32(11)
            y ^= (y << np.uint32(7)) & np.uint32(0x9D2C5680)
            y ^= (y << np.uint32(15)) & np.uint32(0xEFC60000)
            y ^= y >> np.uint32(18)
            out[o:o + t] = y
            o += t
            self.idx += t
        return out


def std_shuffle_minstd(n, seed):
    """std::shuffle(iota(n)) with std::default_random_engine(seed) as libstdc++ 11 implements it."""
    M = 2147483647
    x = seed % M or 1
    URNG = 2147483645   # minstd_rand0: max() - min()

    def g():
        nonlocal x
        x = (16807 * x) % M
        return x

    def uid(a, b):
        urange = b - a
        if URNG > urange:
            uer = urange + 1
            scaling = URNG // uer
            past = uer * scaling
            while True:
                r = g() - 1
                if r < past:
                    return r // scaling + a
        assert URNG == urange
        return g() - 1 + a

    arr = list(range(n))
    if n == 0:
        return np.zeros(0, np.int64)
    if URNG // n >= n:
        i = 1
        if n % 2 == 0:
            j = uid(0, 1)
            arr[i], arr[j] = arr[j], arr[i]
            i += 1
        while i != n:
            sr = i + 1
            v = uid(0, sr * (sr + 1) - 1)
            p1, p2 = v // (sr + 1), v % (sr + 1)
            arr[i], arr[p1] = arr[p1], arr[i]
            i += 1
            arr[i], arr[p2] = arr[p2], arr[i]
            i += 1
    else:
        for i in range(1, n):
            j = uid(0, i)
            arr[i], arr[j] = arr[j], arr[i]
    return np.array(arr, np.int64)


def _symmetric_pattern(n, cp, ir):
    import scipy.sparse as sp
    A = sp.csc_matrix((np.ones(len(ir)), np.asarray(ir, np.int64), np.asarray(cp, np.int64)), shape=(n, n))
    A = A - sp.diags(A.diagonal())
    A.eliminate_zeros()
    B = ((A != 0).astype(np.int8) + (A.T != 0).astype(np.int8)).tocsc()
    B.sort_indices()
    return B


def _nbr_min(B, v, none):
    """out[i] = min over neighbours j of v[j] (none where no neighbour has a value)."""
    out = np.full(B.shape[0], none, v.dtype)
    if B.nnz:
        nz = np.diff(B.indptr) > 0
        out[nz] = np.minimum.reduceat(v[B.indices], B.indptr[:-1][nz])
    return out


def restriction_op(n, cp, ir, mt_seed=1, perm_seed=1383098845):
    """(nagg, colptr, rows, vals, stats) of the reference's R (n x nagg) for the square matrix (cp, ir)."""
    B = _symmetric_pattern(n, cp, ir)
    mt = MT19937(mt_seed)
    NONE = np.uint64(1 << 40)   # above every uint32 draw ("2.0" of RestrictionOp.h:152, 161)
    cand = np.ones(n, bool)
    mis = np.zeros(n, bool)
    rounds = 0
    while cand.any():
        rounds += 1
        r = np.full(n, NONE, np.uint64)
        r[cand] = mt.randint(int(cand.sum())).astype(np.uint64)
        m1 = _nbr_min(B, r, NONE)
        m2 = _nbr_min(B, m1, NONE)
        new = cand & (r <= np.minimum(m1, m2))
        cand &= ~new
        nb1 = _nbr_min(B, np.where(new, 0, 1).astype(np.uint64), np.uint64(1)) == 0
        nb2 = _nbr_min(B, np.where(nb1, 0, 1).astype(np.uint64), np.uint64(1)) == 0
        cand &= ~(nb1 | nb2)
        mis |= new
    # parents: the MIS-2 neighbour (there is at most one), else the vertex itself if it is in the set
    BIG = np.int64(1 << 62)
    parent = _nbr_min(B, np.where(mis, np.arange(n, dtype=np.int64), BIG), BIG)
    parent = np.where(mis, np.arange(n, dtype=np.int64), parent)
    has = parent != BIG
    prob = np.full(n, NONE, np.uint64)
    prob[has] = mt.randint(int(has.sum())).astype(np.uint64)
    # unparented vertices: the parent of the neighbour with the smallest draw; ties -> larger neighbour id
    key = np.where(has, (prob << np.uint64(23)) | (np.uint64((1 << 23) - 1) - np.arange(n, dtype=np.uint64)),
                   np.uint64(2 ** 64 - 1))
    assert n < (1 << 23), "the restatement's tie key packs the vertex id into 23 bits"
    best = _nbr_min(B, key, np.uint64(2 ** 64 - 1))
    nbr = ((1 << 23) - 1) - (best & np.uint64((1 << 23) - 1)).astype(np.int64)
    root = np.where(has, parent, np.where(best != np.uint64(2 ** 64 - 1), parent[np.clip(nbr, 0, n - 1)], -1))
    assert (root >= 0).all(), "MIS-2 aggregation left a vertex without an aggregate"
    misv = np.flatnonzero(mis)
    nagg = len(misv)
    col0 = np.searchsorted(misv, root)   # the parent's rank among the MIS-2 vertices
    perm = std_shuffle_minstd(nagg, perm_seed)
    inv = np.empty(nagg, np.int64)
    inv[perm] = np.arange(nagg)
    col = inv[col0]
    order = np.lexsort((np.arange(n), col))
    rcp = np.zeros(nagg + 1, np.int64)
    np.cumsum(np.bincount(col, minlength=nagg), out=rcp[1:])
    return nagg, rcp, order.astype(np.int64), np.ones(n), {"rounds": rounds, "mis": nagg}
