#!/usr/bin/env python3
"""Every rank's share of the 2/4/8-GPU layouts (1x1x2, 2x2, 2x2x2) for BASELINE configs 4 and 5, at full
size on one GPU -- the real-valued counterparts of `bench.py --rank-share` (R-MAT, multiplicity values).

  config 4  HipMCL expansion A*A of the protein-similarity-like graph (combblas_amd.inputs, n = 2^20 by default)
  config 5  Galerkin R^T A then (R^T A) R: A = 3D Poisson 7-point on k^3 (k = 128), R = the reference's
            RestrictionOp (device), as RestrictionOp.cpp:188-196 multiplies

Rank (l, i, j) gets the panels the panel schedule's broadcasts deliver: A(rows_i, K_l) and B(K_l, cols_j), K_l the
layer-l part of every inner block; with two layers it multiplies the other layer's column half, runs the production
fiber codec on that message (cbg_fiber_codec: the bytes on the link, bit-exact round trip), multiplies its own half,
and merges with the partner's message (the partner's product of this half, made here).  The merged piece is checked
against a one-GPU product A(rows_i, :) * B(:, J_sample) of a seeded column sample: identical structure, values within
1e-12 of the |A| * |B| bound (PlusTimes<double>: accumulation order differs), plus the symbolic pass's nnz of the
whole piece.  One JSON line per (config, N, rank); tools/predict_scaling.py turns them into step predictions.
usage: python tools/rank_share_configs.py [--configs 4,5] [--gpus 2,4,8] [--mcl-n N] [--poisson-k K]"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="4,5")
    ap.add_argument("--gpus", default="2,4,8")
    ap.add_argument("--mcl-n", type=int, default=1 << 20)
    ap.add_argument("--poisson-k", type=int, default=128)
    ap.add_argument("--chunks", type=int, default=int(os.environ.get("CBG_FIBER_CHUNKS", "2")))
    args = ap.parse_args()
    import tempfile
    import torch
    import torch.distributed as dist
    import combblas_amd as cb
    from combblas_amd import dist as cbd
    from combblas_amd.inputs import poisson3d, protein_like_graph
    import bench

    store = tempfile.NamedTemporaryFile(delete=False)
    dist.init_process_group("gloo", init_method=f"file://{store.name}", rank=0, world_size=1)
    ctx = cb.Context(0)
    be = cbd.GpuBackend(ctx)
    SR = cb.PlusTimesSRing("f64")
    dev = be.device

    def host_block(M, r0, r1, c0, c1):
        nrow, ncol, cp, ir, val = M
        lcp, lir, lval = cbd.slice_csc(cp, ir, val, r0, r1, c0, c1)
        return cbd.block_from_host(r1 - r0, c1 - c0, lcp, lir, lval, dev)

    def panels(Am, Bm, q, L, l, i, j):
        """A(rows_i, K_l) (pieces side by side) and B(K_l, cols_j) (pieces stacked): the panel schedule's operands."""
        kin = Am[1]
        r0, r1 = cbd.block_range(Am[0], q, i)
        c0, c1 = cbd.block_range(Bm[1], q, j)
        ks = [cbd.piece_range(kin, q, L, k, l) for k in range(q)]
        AP = bench._hcat([host_block(Am, r0, r1, k0, k1) for (k0, k1) in ks])
        BP = bench._vstack([host_block(Bm, k0, k1, c0, c1) for (k0, k1) in ks])
        return AP, BP

    def abs_block(b):
        return cbd.Block(b.nrow, b.ncol, b.cp, b.ir, b.val.abs())

    def check(M, Am, Bm, r0, r1, c0, c1, nsample, seed):
        """The rank's merged piece against an independent one-GPU product of sampled columns."""
        Arow = host_block(Am, r0, r1, 0, Am[1])
        Bcol = host_block(Bm, 0, Bm[0], c0, c1)
        est_m, est_z = be.estimate(Arow, Bcol)
        k = min(M.ncol, int(nsample))
        g = torch.Generator().manual_seed(int(seed))
        sel = torch.randperm(M.ncol, generator=g)[:k].sort().values
        Bs = bench.select_block_cols(Bcol, sel)
        P = be.multiply(Arow, Bs, SR)
        Pabs = be.multiply(abs_block(Arow), abs_block(Bs), SR)
        S = bench.select_block_cols(M, sel)
        same = P.nnz == S.nnz and torch.equal(P.cp, S.cp) and torch.equal(P.ir, S.ir)
        err = float(((P.val - S.val).abs() / torch.clamp(Pabs.val, min=1e-300)).max().item()) if same and P.nnz else 0.0
        rec = {"sampled_columns": k, "sample_nnz": P.nnz, "structure_equal": bool(same),
               "max_rel_err_vs_abs_bound": err, "within_1e-12": bool(same and err <= 1e-12),
               "piece_nnz": M.nnz, "piece_nnz_equals_estimate": M.nnz == est_z, "piece_multiplies_estimate": est_m}
        rec.update(oracle_check(M, Arow, Bcol, 256, seed))
        rec["within_1e-12"] = rec["within_1e-12"] and rec["oracle_sample"]
        return rec

    def oracle_check(M, Arow, Bcol, ncols, seed):
        """CHECKER (test infrastructure): 256 seeded columns of the piece against oracle/oracle.c's product on the host
        (the reference-pinned restatement of LocalSpGEMMHash), structure exact, values within 1e-12 of |A|*|B|."""
        sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests"))
        from helpers import Csc, oracle_spgemm
        k = min(M.ncol, int(ncols))
        g = torch.Generator().manual_seed(int(seed) ^ 0x5EED)
        sel = torch.randperm(M.ncol, generator=g)[:k].sort().values
        Bs = bench.select_block_cols(Bcol, sel)
        S = bench.select_block_cols(M, sel)
        h = lambda b, f=lambda v: v: Csc(b.nrow, b.ncol, b.cp.cpu().numpy(), b.ir.cpu().numpy(), f(b.val.cpu().numpy()))
        R, _, rc = oracle_spgemm(h(Arow), h(Bs), "plus_times", "f64")
        Ra, _, rca = oracle_spgemm(h(Arow, np.abs), h(Bs, np.abs), "plus_times", "f64")
        same = (rc == 0 and rca == 0 and np.array_equal(S.cp.cpu().numpy(), R.cp)
                and np.array_equal(S.ir.cpu().numpy(), R.ir))
        err = float(np.max(np.abs(S.val.cpu().numpy() - R.val) / np.maximum(Ra.val, 1e-300))) if same and len(R.val) else 0.0
        return {"oracle_sample_columns": k, "oracle_sample_nnz": int(R.cp[-1]), "oracle_max_rel_err": err,
                "oracle_sample": bool(same and err <= 1e-12)}

    def prune_share(M, Am, Bm, q, i, b0, h0, h1):
        """configs[3]: the rank's part of the distributed MCLPruneRecoverySelect (ParFriends.h:185-353, MCL.cpp:573-587).
        With q = 1 the piece holds complete columns and is pruned as is; with q > 1 the rank prunes column group i of
        its piece's columns, completed along the processor column (dist._gather_columns: rows of all q row blocks),
        built here as one product A * B(:, group).  Records the prune time and the gathered entries."""
        d = cb.MCL_DEFAULTS
        if q == 1:
            full = M
            gathered = 0
        else:
            g0, g1 = cbd.block_range(h1 - h0, q, i)
            full = be.multiply(host_block(Am, 0, Am[0], 0, Am[1]), host_block(Bm, 0, Bm[0], b0 + h0 + g0, b0 + h0 + g1), SR)
            gathered = int(full.nnz)
        ts = []
        for rep in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            P, stp = be.mcl_prune(full, d["hardThreshold"], d["selectNum"], d["recoverNum"], d["recoverPct"])
            torch.cuda.synchronize()
            ts.append(1e3 * (time.perf_counter() - t0))
            kept = int(P.nnz)
            del P
        rec = {"prune_ms": round(ts[-1], 3), "prune_columns": int(full.ncol), "prune_in_nnz": int(full.nnz),
               "prune_kept_nnz": kept, "gathered_entries": gathered,
               "gather_bytes_offrank": int(gathered * 12 * (q - 1) / q) if q > 1 else 0, **stp}
        del full
        torch.cuda.empty_cache()
        return rec

    def run(label, Am, Bm, N, extra):
        L, q, _ = cbd.grid_for(N)
        bad = False
        for r in range(N):
            l, rem = divmod(r, q * q)
            i, j = divmod(rem, q)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            AP, BP = panels(Am, Bm, q, L, l, i, j)
            build_s = time.perf_counter() - t0
            nc = BP.ncol
            halves = [cbd.block_range(nc, L, m) for m in range(L)]
            me, other = (l, 1 - l) if L == 2 else (0, None)
            rec = {"config": label, "rank": r, "layout": f"{L}x{q}x{q}", "l_i_j": [l, i, j], **extra,
                   "nnz_A_panel": AP.nnz, "nnz_B_panel": BP.nnz, "panel_build_s": round(build_s, 3)}
            gather = False
            if L == 2:   # the grid's choice (grid.hip fiber_gather_ok): the partial's multiplies vs the entries to send
                Bo = bench._col_slice_block(BP, *halves[other])
                flops_other = int(torch.diff(AP.cp)[Bo.ir.to(torch.int64)].sum().item()) if Bo.nnz else 0
                gather = flops_other >= 4.0 * (AP.nnz + Bo.nnz)
                if gather:
                    PA, PB = panels(Am, Bm, q, L, other, i, j)
                    mine_b = bench._col_slice_block(BP, *halves[me])
                    part_b = bench._col_slice_block(PB, *halves[me])
                    rec["gather_bytes_sent"] = 12 * (AP.nnz + Bo.nnz) + 8 * (AP.ncol + Bo.ncol + 2)
                    rec["gather_bytes_recv"] = 12 * (PA.nnz + part_b.nnz) + 8 * (PA.ncol + part_b.ncol + 2)
                    A2 = bench._hcat([AP, PA] if me == 0 else [PA, AP])
                    B2 = bench._vstack([mine_b, part_b] if me == 0 else [part_b, mine_b])
                    del PA, PB, mine_b, part_b
                del Bo
            rec["fiber_mode"] = "gather" if gather else ("reduce" if L == 2 else "none")
            for rep in range(2):   # the second repetition is recorded
                st = {}
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                if gather:
                    M = be.multiply(A2, B2, SR, st)
                    torch.cuda.synchronize()
                    local_ms, merge_ms, codec = 1e3 * (time.perf_counter() - t0), 0.0, None
                    profs = [ctx.last_profile()]
                elif L == 2:
                    Po = be.multiply(AP, bench._col_slice_block(BP, *halves[other]), SR, st)
                    t1 = time.perf_counter()
                    p_other = ctx.last_profile()
                    codec = be.fiber_codec(Po, args.chunks) if rep == 1 else None
                    del Po
                    torch.cuda.synchronize()
                    t2 = time.perf_counter()
                    Pm = be.multiply(AP, bench._col_slice_block(BP, *halves[me]), SR, st)
                    t3 = time.perf_counter()
                    p_mine = ctx.last_profile()
                    PA, PB = panels(Am, Bm, q, L, other, i, j)
                    Pr = be.multiply(PA, bench._col_slice_block(PB, *halves[me]), SR)
                    del PA, PB
                    torch.cuda.synchronize()
                    t4 = time.perf_counter()
                    M = be.merge([Pm, Pr] if me == 0 else [Pr, Pm], SR)
                    torch.cuda.synchronize()
                    t5 = time.perf_counter()
                    local_ms, merge_ms = 1e3 * ((t1 - t0) + (t3 - t2)), 1e3 * (t5 - t4)
                    rec["recv_nnz"] = Pr.nnz
                    profs = [p_other, p_mine]
                    del Pm, Pr
                else:
                    M = be.multiply(AP, BP, SR, st)
                    torch.cuda.synchronize()
                    local_ms, merge_ms, codec = 1e3 * (time.perf_counter() - t0), 0.0, None
                    profs = [ctx.last_profile()]
                final = M if rep == 1 else None
                del M
                torch.cuda.empty_cache()
            del AP, BP
            if gather:
                del A2, B2
            r0, r1 = cbd.block_range(Am[0], q, i)
            b0, _ = cbd.block_range(Bm[1], q, j)
            h0, h1 = halves[me]
            v = check(final, Am, Bm, r0, r1, b0 + h0, b0 + h1, max(int(np.ceil(1e4 / N)), final.ncol // 64),
                      7919 * r + 11)
            if label.startswith("4"):
                rec["prune"] = prune_share(final, Am, Bm, q, i, b0, h0, h1)
            del final
            torch.cuda.empty_cache()
            rec.update({"multiplies": st.get("multiplies", 0), "local_ms": round(local_ms, 3),
                        "merge_ms": round(merge_ms, 3), "verified": v,
                        "phases_ms": [{k: round(float(pp[k]), 3) for k in
                                       ("flops_ms", "bin_ms", "symbolic_ms", "scan_ms", "numeric_ms", "heavy_ms",
                                        "total_ms")} for pp in profs],
                        "fiber_codec": codec,
                        "fiber": None if codec is None else {"bytes": codec["wire_bytes"],
                                                            "bytes_per_entry": round(codec["wire_bytes"] /
                                                                                     max(codec["entries"], 1), 3)}})
            print(json.dumps(rec), flush=True)
            bad = bad or not (v["within_1e-12"] and v["piece_nnz_equals_estimate"]
                              and (codec is None or codec["roundtrip_exact"]))
        return bad

    def anchor4(Am, extra):
        """configs[3] at N = 1 on the same graph: the expansion product and MCLPruneRecoverySelect on one GPU (the
        denominator of the 2/4/8-GPU predictions), the prune's kept entries against the oracle's prune on a sample."""
        A = host_block(Am, 0, Am[0], 0, Am[1])
        d = cb.MCL_DEFAULTS
        rec = {"config": "4: HipMCL expansion A*A", "rank": 0, "layout": "1 GPU", **extra}
        for rep in range(2):
            st = {}
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            C = be.multiply(A, A, SR, st)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            P, stp = be.mcl_prune(C, d["hardThreshold"], d["selectNum"], d["recoverNum"], d["recoverPct"])
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            prof = ctx.last_profile()
            nnz_c, nnz_p = C.nnz, P.nnz
            if rep == 0:
                del P
            del C
            torch.cuda.empty_cache()
        mults = st.get("multiplies", 0)
        rec.update({"multiplies": mults, "local_ms": round(1e3 * (t1 - t0), 3), "prune_ms": round(1e3 * (t2 - t1), 3),
                    "expansion_ms": round(1e3 * (t2 - t0), 3), "nnz_C": nnz_c, "nnz_pruned": nnz_p, **stp,
                    "multiplies_per_s_expansion": mults / (t2 - t0), "merge_ms": 0.0, "fiber": None,
                    "nnz_A_panel": A.nnz, "nnz_B_panel": A.nnz})
        # the pruned columns of a seeded sample against the oracle's MCLPruneRecoverySelect of the same columns
        sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests"))
        from helpers import Csc, oracle_spgemm, oracle_mcl_prune
        g = torch.Generator().manual_seed(4242)
        sel = torch.randperm(A.ncol, generator=g)[:256].sort().values
        Bs = bench.select_block_cols(A, sel)
        h = lambda b: Csc(b.nrow, b.ncol, b.cp.cpu().numpy(), b.ir.cpu().numpy(), b.val.cpu().numpy())
        R, _, rc = oracle_spgemm(h(A), h(Bs), "plus_times", "f64")
        O = oracle_mcl_prune(R, d["hardThreshold"], d["selectNum"], d["recoverNum"], d["recoverPct"])
        S = bench.select_block_cols(P, sel)
        ok = rc == 0 and np.array_equal(S.cp.cpu().numpy(), O[0].cp) and np.array_equal(S.ir.cpu().numpy(), O[0].ir)
        rec["verified"] = {"oracle_prune_sample_columns": 256, "oracle_prune_structure_equal": bool(ok),
                           "oracle_prune_sample_nnz": int(O[0].cp[-1])}
        del P
        torch.cuda.empty_cache()
        print(json.dumps(rec), flush=True)
        return not ok

    bad = False
    gpus = [int(x) for x in args.gpus.split(",")]
    for c in [int(x) for x in args.configs.split(",")]:
        if c == 4:
            t0 = time.perf_counter()
            n, cp, ir, val = protein_like_graph(args.mcl_n, seed=1)
            A = (n, n, cp, ir, val)
            extra = {"graph_n": n, "nnz": int(cp[-1]), "gen_s": round(time.perf_counter() - t0, 1)}
            for N in gpus:
                if N == 1:
                    bad |= anchor4(A, extra)
                else:
                    bad |= run("4: HipMCL expansion A*A", A, A, N, extra)
        elif c == 5:
            n, acp, air, aval = poisson3d(args.poisson_k)
            dA = cb.SpDCCols.from_csc(ctx, n, n, acp, air, aval)
            dR, dRt = cb.RestrictionOp(dA)
            R = (n, dR.getncol()) + tuple(dR.to_host())
            Rt = (dRt.getnrow(), n) + tuple(dRt.to_host())
            RA = cb.LocalSpGEMMHash(SR, dRt, dA)
            RAh = (RA.getnrow(), n) + tuple(RA.to_host())
            for m in (dA, dR, dRt, RA):
                m.free()
            A = (n, n, acp, air, aval)
            extra = {"poisson_k": args.poisson_k, "n": n, "nagg": R[1]}
            for N in gpus:
                bad |= run("5a: Galerkin R^T A", Rt, A, N, extra)
                bad |= run("5b: Galerkin (R^T A) R", RAh, R, N, extra)
    dist.destroy_process_group()
    if os.path.exists(store.name):
        os.unlink(store.name)
    if bad:
        sys.exit("rank_share_configs: a piece failed its checks")


if __name__ == "__main__":
    main()
