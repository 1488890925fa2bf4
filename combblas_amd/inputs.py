"""Synthetic inputs of BASELINE configs 4 and 5 (host side, numpy; deterministic in `seed`).

* protein_like_graph: HipMCL-style similarity graph (config 4) -- planted clusters with log-uniform
  sizes, intra-cluster density, inter-cluster noise, symmetric weights uniform(0.1, 1], self loops
  (MCL's AddLoops, Applications/MCL.cpp), made column stochastic (MakeColStochastic, MCL.cpp:390).
* poisson3d: 7-point Laplacian on a k^3 grid (diag 6, off-diagonal -1), the A of the Galerkin triple
  product (config 5; 3DSpGEMM/RestrictionOp.cpp drives R^T A R).
* aggregation_restriction: the restriction operator R (n x nagg, one 1 per row) of a distance-2
  maximal-independent-set aggregation (RestrictionOp.h:116-427: MIS-2 roots, every vertex joins the
  aggregate of a root within distance 2).  Our MIS-2 runs Luby-style rounds on seeded random
  priorities (vectorised); the reference's distributed MIS-2 draws its own priorities, so R is a
  valid aggregation of the same kind, not the reference's bit pattern (config 5 parity is about the
  R^T A R product, checked against the reference and the oracle on identical R).
All return host CSC arrays (int64 colptr, int32 rows, float64 values).
"""
import numpy as np


def _csc_from_coo(nrow, ncol, r, c, v, dup="sum"):
    import scipy.sparse as sp
    M = sp.coo_matrix((v, (r, c)), shape=(nrow, ncol)).tocsc()
    M.sum_duplicates()
    M.sort_indices()
    return M.indptr.astype(np.int64), M.indices.astype(np.int32), M.data.astype(np.float64)


def protein_like_graph(n, seed=1, cmin=20, cmax=2000, density=0.2, noise=1e-5):
    """(n, colptr, rows, vals): column-stochastic planted-cluster graph (BASELINE config 4)."""
    rng = np.random.default_rng(seed)
    sizes, tot = [], 0
    cmax = max(cmin, min(cmax, n))
    while tot < n:
        s = int(np.exp(rng.uniform(np.log(cmin), np.log(cmax))))
        s = max(1, min(s, n - tot))
        sizes.append(s)
        tot += s
    perm = rng.permutation(n).astype(np.int64)
    R, C = [], []
    start = 0
    for s in sizes:
        pairs = s * (s - 1) // 2
        m = int(rng.binomial(pairs, density)) if pairs else 0
        if m:
            a = rng.integers(0, s, size=m)
            b = rng.integers(0, s, size=m)
            keep = a != b
            R.append(start + np.minimum(a, b)[keep])
            C.append(start + np.maximum(a, b)[keep])
        start += s
    m_noise = int(noise * n * (n - 1) / 2)
    if m_noise:
        a = rng.integers(0, n, size=m_noise)
        b = rng.integers(0, n, size=m_noise)
        keep = a != b
        R.append(np.minimum(a, b)[keep])
        C.append(np.maximum(a, b)[keep])
    r = np.concatenate(R) if R else np.zeros(0, np.int64)
    c = np.concatenate(C) if C else np.zeros(0, np.int64)
    key = np.unique(r * n + c)
    r, c = key // n, key % n
    w = rng.uniform(0.1, 1.0, size=len(r))
    w = np.where(w <= 0.1, 1.0, w)   # (0.1, 1]
    rr = perm[np.concatenate([r, c, np.arange(n)])]
    cc = perm[np.concatenate([c, r, np.arange(n)])]
    vv = np.concatenate([w, w, np.ones(n)])
    cp, ir, val = _csc_from_coo(n, n, rr, cc, vv)
    colsum = np.add.reduceat(val, cp[:-1]) if len(val) else np.zeros(n)
    val = val / np.repeat(colsum, np.diff(cp))
    return n, cp, ir, val


def poisson3d(k):
    """(n, colptr, rows, vals) of the 7-point Laplacian on a k x k x k grid (n = k^3)."""
    n = k ** 3
    idx = np.arange(n, dtype=np.int64)
    x, y, z = idx % k, (idx // k) % k, idx // (k * k)
    rows, cols, vals = [idx], [idx], [np.full(n, 6.0)]
    for d, coord, stride in ((1, x, 1), (1, y, k), (1, z, k * k)):
        m = coord < k - 1
        a, b = idx[m], idx[m] + stride
        rows += [a, b]
        cols += [b, a]
        vals += [np.full(len(a), -1.0), np.full(len(a), -1.0)]
    cp, ir, val = _csc_from_coo(n, n, np.concatenate(rows), np.concatenate(cols), np.concatenate(vals))
    return n, cp, ir, val


def mis_keys(n, seed):
    """Distinct nonzero 64-bit priorities of vertices 0..n-1 (the device's mis_key, galerkin.hip): a
    seeded splitmix64 hash in the high 32 bits, the vertex id in the low 32 bits, plus one."""
    M = (1 << 64) - 1
    v = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = v ^ np.uint64((seed * 0x9E3779B97F4A7C15) & M)
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
        return ((z >> np.uint64(32)) << np.uint64(32) | v) + np.uint64(1)


def aggregation_restriction(n, cp, ir, seed=1):
    """(nagg, colptr, rows, vals) of R (n x nagg): MIS-2 aggregation of the graph of a symmetric CSC,
    the shape RestrictionOp.h:116-290 builds; host restatement of cbg_mis2_restriction (galerkin.hip),
    same priorities (mis_keys), same rounds, same aggregate numbering.  Luby rounds: an undecided vertex
    whose key is the largest among the undecided vertices within distance 2 becomes a root, and its
    distance-2 neighbourhood is decided; then every vertex joins the highest-key root within distance 1,
    else within distance 2.  R[i, agg(i)] = 1; aggregates numbered in root-vertex order."""
    import scipy.sparse as sp
    G = sp.csr_matrix((np.ones(len(ir)), ir, cp), shape=(n, n))
    G = G + sp.identity(n, format="csr")
    G2 = (G @ G).tocsr()
    G.sort_indices()
    G2.sort_indices()
    prio = mis_keys(n, seed)
    state = np.zeros(n, np.int8)                        # 0 undecided, 1 root, 2 covered

    def rowmax(M, v):
        out = np.zeros(M.shape[0], np.uint64)
        nz = np.diff(M.indptr) > 0
        if M.nnz:
            out[nz] = np.maximum.reduceat(v[M.indices], M.indptr[:-1][nz])
        return out

    while (state == 0).any():
        p = np.where(state == 0, prio, np.uint64(0))
        m2 = rowmax(G2, p)
        new = (state == 0) & (p == m2)
        state[new] = 1
        covered = (G2 @ new.astype(np.float64)) > 0
        state[(state == 0) & covered] = 2
    isroot = state == 1
    rid = np.cumsum(isroot) - isroot                    # root ids in vertex order
    rp = np.where(isroot, prio, np.uint64(0))
    agg = np.full(n, -1, np.int64)
    for M in (G, G2):                                   # nearest: distance 1, then 2
        best = rowmax(M, rp)
        undone = (agg < 0) & (best > 0)
        agg[undone] = rid[((best[undone] - np.uint64(1)) & np.uint64(0xFFFFFFFF)).astype(np.int64)]
    assert (agg >= 0).all()
    nagg = int(isroot.sum())
    rcp, rir, rval = _csc_from_coo(n, nagg, np.arange(n), agg, np.ones(n))
    return nagg, rcp, rir, rval
