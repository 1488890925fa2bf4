#!/usr/bin/env python3
"""Anatomy of the heavy-column work at an R-MAT scale (CPU only, sampled): how many A entries the
heavy units gather versus the useful multiplies, and how many (unit, B nonzero) segments they stage.

    python tools/heavy_anatomy.py [scale] [sample_columns]

Mirrors the unit formation of k_build_units (spgemm_kernels.hpp): subwindows of SUBW rows, units of
consecutive subwindows with <= UNIT_CAP outputs and a span <= SPAN_CAP rows; an A column of at least
SPLIT_MIN entries contributes only its rows inside the unit (split table), a shorter one is read whole
by every unit its row range intersects (rows outside are dropped at insert).
"""
import os
import sys

import numpy as np
import scipy.sparse as sp

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

K_HEAVY, UNIT_CAP, SPAN_CAP, SPLIT_MIN, NT = 4096, 6144, 458752, 16, 1024


def main():
    scale = int(sys.argv[1]) if len(sys.argv) > 1 else 18
    ns = int(sys.argv[2]) if len(sys.argv) > 2 else 400
    import combblas_amd as cb
    n, cp, ir, val = cb.generate_rmat_host(scale, 16, seed=1)
    A = sp.csc_matrix((np.ones(len(ir)), ir, cp), shape=(n, n))
    slog = 13
    while ((n - 1) >> slog) + 1 > 2048:
        slog += 1
    alen = np.diff(cp)
    flop = np.bincount(np.repeat(np.arange(n), alen), weights=alen[ir], minlength=n)
    # heavy candidates: flop > K_HEAVY (nnz(C) > K_HEAVY implies it); sample weighted by flop
    cand = np.nonzero(flop > K_HEAVY)[0]
    rng = np.random.default_rng(0)
    pick = np.sort(rng.choice(cand, size=min(ns, len(cand)), replace=False))
    C = (A @ A[:, pick]).tocsc()
    C.sort_indices()
    tot = dict(mult=0, gathered=0, segs=0, nonempty=0, units=0, chunks=0, nnzc=0, heavy=0, nb=0)
    hist = np.zeros(66, np.int64)   # nonempty segment lengths (64+ pooled in the last bin)
    dens = np.zeros(12)             # multiplies of units by span/cnt ratio bucket (log2)
    first = np.where(alen > 0, ir[np.minimum(cp[:-1], len(ir) - 1)], 0)
    last = np.where(alen > 0, ir[np.maximum(cp[1:] - 1, 0)], -1)
    for t, j in enumerate(pick):
        rows = C.indices[C.indptr[t]:C.indptr[t + 1]]
        if len(rows) <= K_HEAVY:
            continue
        tot["heavy"] += 1
        sub = np.bincount(rows >> slog, minlength=((n - 1) >> slog) + 1)
        sf, sl = rows[0] >> slog, rows[-1] >> slog
        units, st, acc = [], sf, 0
        for s in range(sf, sl + 1):
            wide = ((s + 1 - st) << slog) > SPAN_CAP
            if acc > 0 and (acc + sub[s] > UNIT_CAP or wide):
                units.append((st, s))
                st, acc = s, 0
            acc += sub[s]
        if acc > 0:
            units.append((st, sl + 1))
        ks = ir[cp[j]:cp[j + 1]]
        nb = len(ks)
        tot["nb"] += nb
        tot["units"] += len(units)
        tot["nnzc"] += len(rows)
        tot["mult"] += int(alen[ks].sum())
        tot["chunks"] += len(units) * ((nb + NT - 1) // NT)
        for (s0, s1) in units:
            r0, r1 = s0 << slog, s1 << slog
            ucnt = int(((rows >= r0) & (rows < r1)).sum())
            ulo, uhi = max(r0, int(rows[0])), min(r1 - 1, int(rows[-1]))
            umult = 0
            longk = alen[ks] >= SPLIT_MIN
            # long columns: exact pieces
            lk = ks[longk]
            if len(lk):
                a_lo = np.array([np.searchsorted(ir[cp[k]:cp[k + 1]], r0) for k in lk])
                a_hi = np.array([np.searchsorted(ir[cp[k]:cp[k + 1]], r1) for k in lk])
                g = a_hi - a_lo
                tot["gathered"] += int(g.sum())
                umult += int(g.sum())
                tot["nonempty"] += int((g > 0).sum())
                hist += np.bincount(np.minimum(g[g > 0], 65), minlength=66)
            sk = ks[~longk]
            hit = (last[sk] >= r0) & (first[sk] < r1) & (alen[sk] > 0)
            tot["gathered"] += int(alen[sk][hit].sum())
            tot["nonempty"] += int(hit.sum())
            hist += np.bincount(np.minimum(alen[sk][hit], 65), minlength=66)
            tot["segs"] += nb
            if ucnt > 0:
                dens[min(11, int(np.log2(max(1.0, (uhi - ulo + 1) / ucnt))))] += umult
    h = tot["heavy"]
    print(f"scale {scale}: {len(cand)} flop-heavy candidate columns, sampled {len(pick)}, heavy {h}")
    for k, v in tot.items():
        print(f"  {k:10s} {v:14d}  per heavy column {v / max(h, 1):12.1f}")
    print(f"  gathered / useful multiplies = {tot['gathered'] / max(tot['mult'], 1):.3f}")
    print(f"  staged segments / multiply   = {tot['segs'] / max(tot['mult'], 1):.3f}   "
          f"nonempty / staged = {tot['nonempty'] / max(tot['segs'], 1):.3f}")
    print("  multiplies by unit span/cnt (log2 bucket):", [round(float(x / max(dens.sum(), 1)), 3) for x in dens])
    L = np.arange(66)
    print("  nonempty segment lengths:", {int(l): round(float(hist[l] / max(hist.sum(), 1)), 4) for l in L if hist[l]})
    for G in (1, 2, 4, 8):
        groups = int((hist * ((L + G - 1) // G)).sum())
        print(f"  G={G}: groups {groups}, gathered/group {tot['gathered'] / max(groups, 1):.2f} (fill {tot['gathered'] / max(groups * G, 1):.2f})")
    print(f"  multiplies per unit = {tot['mult'] / max(tot['units'], 1):.0f}, outputs per unit = "
          f"{tot['nnzc'] / max(tot['units'], 1):.0f}, chunks per unit = {tot['chunks'] / max(tot['units'], 1):.2f}")


if __name__ == "__main__":
    main()
