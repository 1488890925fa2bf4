#!/usr/bin/env python3
"""Anatomy of the heavy-column work at an R-MAT scale (CPU only, sampled): how many A entries the
heavy units gather versus the useful multiplies, and how many (unit, B nonzero) segments they stage.

    python tools/heavy_anatomy.py [scale] [sample_columns] [nrow_panel_log]

The second section is k_sym_part's view: every wide column is swept once per 2^18-row part, each B nonzero
staging one segment (its A column narrowed to the part by the part table); the histogram of the non-empty segment
lengths says how many vec4 groups and gather lines one part costs.  nrow_panel_log (e.g. 21) restricts A to the
rows of one 2x2x2 rank panel (the s22 rank-share size: 2^21 rows), as the per-rank product sees it.

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

K_HEAVY, UNIT_CAP, SPAN_CAP, SPLIT_MIN, NT = 4096, 7168, 458752, 16, 1024


def main():
    scale = int(sys.argv[1]) if len(sys.argv) > 1 else 18
    ns = int(sys.argv[2]) if len(sys.argv) > 2 else 400
    import combblas_amd as cb
    n, cp, ir, val = cb.generate_rmat_host(scale, 16, seed=1)
    A = sp.csc_matrix((np.ones(len(ir)), ir, cp), shape=(n, n))
    Bfull = A
    if len(sys.argv) > 3:   # one rank panel: A(rows 0 .. 2^p - 1, :) times columns of the whole matrix
        nr = 1 << int(sys.argv[3])
        A = A[:nr, :].tocsc()
        A.sort_indices()
        cp, ir = A.indptr.astype(np.int64), A.indices.astype(np.int64)
    slog = 13
    while ((n - 1) >> slog) + 1 > 2048:
        slog += 1
    alen = np.diff(cp)
    bcp, bir = Bfull.indptr.astype(np.int64), Bfull.indices.astype(np.int64)
    flop = np.bincount(np.repeat(np.arange(n), np.diff(bcp)), weights=alen[bir], minlength=n)
    # heavy candidates: flop > K_HEAVY (nnz(C) > K_HEAVY implies it); sample weighted by flop
    cand = np.nonzero(flop > K_HEAVY)[0]
    rng = np.random.default_rng(0)
    pick = np.sort(rng.choice(cand, size=min(ns, len(cand)), replace=False))
    C = (A @ Bfull[:, pick]).tocsc()
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
        ks = bir[bcp[j]:bcp[j + 1]]
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
    part_anatomy(A, cp, ir, bcp, bir, pick, C)


def part_anatomy(A, cp, ir, bcp, bir, pick, C, plog=18, G=4):
    """k_sym_part's work per (wide column, part): staged segments (one per B nonzero and part), the non-empty
    ones, their length histogram, vec4 groups and the 64-byte lines the groups touch."""
    nrow = A.shape[0]
    P = ((nrow - 1) >> plog) + 1
    col = np.repeat(np.arange(A.shape[1]), np.diff(cp))
    cnt = np.bincount(col * P + (ir >> plog), minlength=A.shape[1] * P).reshape(A.shape[1], P)
    pos = ir - cp[col]                          # entry's position in its column
    tot = dict(parts=0, staged=0, nonempty=0, mult=0, groups=0, lines=0, outputs=0)
    # word privatisation: the bitmap ORs one LDS instruction issues -- 64 lanes, each on the i-th entry of
    # its group of G consecutive entries of one segment, lanes on consecutive groups -- against the distinct bitmap
    # words among them (what a wave-level combine would issue), and against the distinct words inside each group
    pv = dict(lane_entries=0, words_per_instr=0, words_per_group=0)
    hist = np.zeros(66, np.int64)
    for t, j in enumerate(pick):
        rows = C.indices[C.indptr[t]:C.indptr[t + 1]]
        if len(rows) <= K_HEAVY:
            continue
        ks = bir[bcp[j]:bcp[j + 1]]
        for p in range(rows[0] >> plog, (rows[-1] >> plog) + 1):
            L = cnt[ks, p]
            tot["parts"] += 1
            tot["staged"] += len(ks)
            tot["nonempty"] += int((L > 0).sum())
            tot["mult"] += int(L.sum())
            tot["groups"] += int(((L + G - 1) // G).sum())
            tot["outputs"] += int(((rows >> plog) == p).sum())
            hist += np.bincount(np.minimum(L[L > 0], 65), minlength=66)
            # 64-byte lines: a part's entries of column k start at cp[k] + cnt[k, :p].sum()
            start = cp[ks] + cnt[ks, :p].sum(axis=1)
            nz = L > 0
            tot["lines"] += int((((start[nz] + L[nz] - 1) * 4) // 64 - (start[nz] * 4) // 64 + 1).sum())
            if nz.any():   # this part's multiplies in staging order: segments in B order, rows ascending in each
                segs = [ir[s0:s0 + l] for s0, l in zip(start[nz], L[nz])]
                words = np.concatenate(segs).astype(np.int64) >> 5
                gcnt = (L[nz] + G - 1) // G
                gid = np.concatenate([np.arange(l) // G for l in L[nz]]) + np.repeat(
                    np.concatenate([[0], np.cumsum(gcnt)[:-1]]), L[nz])
                ent = np.concatenate([np.arange(l) % G for l in L[nz]])
                pv["lane_entries"] += len(words)
                key_g = gid * (1 << 40) + words
                pv["words_per_group"] += len(np.unique(key_g))
                key_i = ((gid // 64) * G + ent) * (1 << 40) + words   # (wave step, entry index) -> distinct words
                pv["words_per_instr"] += len(np.unique(key_i))
    del pos
    print(f"k_sym_part view ({P} parts of 2^{plog} rows over {nrow} rows):")
    for k, v in tot.items():
        print(f"  {k:10s} {v:14d}  per part {v / max(tot['parts'], 1):12.1f}")
    print(f"  nonempty / staged = {tot['nonempty'] / max(tot['staged'], 1):.3f}, multiplies / nonempty segment = "
          f"{tot['mult'] / max(tot['nonempty'], 1):.2f}, multiplies / group = {tot['mult'] / max(tot['groups'], 1):.2f}, "
          f"lines / multiply = {tot['lines'] / max(tot['mult'], 1):.3f}, multiplies / output = "
          f"{tot['mult'] / max(tot['outputs'], 1):.2f}")
    Lr = np.arange(66)
    print("  nonempty part-segment lengths:", {int(l): round(float(hist[l] / max(hist.sum(), 1)), 4) for l in Lr if hist[l]})
    e = max(pv["lane_entries"], 1)
    print(f"  word privatisation: bitmap ORs now {pv['lane_entries']} (one per multiply; the read-before-OR skips set "
          f"bits), distinct words per wave instruction {pv['words_per_instr']} ({pv['words_per_instr'] / e:.4f} of them), "
          f"distinct words per lane group {pv['words_per_group']} ({pv['words_per_group'] / e:.4f})")


if __name__ == "__main__":
    main()
