#!/usr/bin/env python3
"""Predicted N-GPU step time of the mandated layouts from the one-GPU rank shares (`bench.py --rank-share`).

Per rank: the panel broadcasts (its A and B panels less the pieces it owns, over one link), then on two-layer grids
either the fiber gather (records with fiber_mode "gather": the partners swap their layer operands over one link, then
one product) or the fiber pipeline -- the other layer's column half multiplied in C chunks, each chunk's message sent as soon as it
is made while the next chunk and then the own half multiply (one link per direction, the partner's message arriving
on the same schedule) -- then the decode of the received message and the merge; one-layer grids multiply once.
The step is the slowest rank's; the value is the multiplies of all ranks over it.  When the record carries the
production codec's measurement (`fiber_codec`, cbg_fiber_codec on the same message), its encode time is added to the
compute stream (the pipeline encodes each chunk between the products) and its decode time replaces the decode model.
A file holding several workloads (tools/rank_share_configs.py) is predicted per (config, layout).

usage: python tools/predict_scaling.py profiles/r04l_rank_share_s22_n8.jsonl [--link-GBps 64] [--chunks 2]
"""
import argparse
import json


def rank_step(rec, link_gbps, chunks, decode_gbps=5000.0, entry_bytes=12, decode_hidden=0.0):
    """Milliseconds of one rank's step (see the module docstring); returns (total, parts)."""
    bw = link_gbps * 1e9 / 1e3   # bytes per ms
    if rec["layout"] == "1 GPU":   # the N = 1 anchor (configs 4: expansion + prune on one GPU)
        t = float(rec["local_ms"]) + float(rec.get("prune_ms", 0.0))
        return t, {"compute": float(rec["local_ms"]), "prune": float(rec.get("prune_ms", 0.0))}
    total, parts = rank_step_grid(rec, link_gbps, chunks, decode_gbps, entry_bytes, decode_hidden)
    pr = rec.get("prune")
    if pr:   # configs 4: the distributed MCLPruneRecoverySelect after the product: the rank's column group gathered
        # along the processor column (its unpruned entries from the q - 1 other row blocks), pruned, and the kept
        # entries scattered back (dist._gather_columns / _scatter_columns)
        q = int(rec["layout"].split("x")[1])
        back = pr.get("prune_kept_nnz", 0) * entry_bytes * (q - 1) / q if pr.get("gather_bytes_offrank") else 0.0
        parts["prune"] = float(pr["prune_ms"]) + (pr.get("gather_bytes_offrank", 0) + back) / bw
        total += parts["prune"]
    return total, parts


def rank_step_grid(rec, link_gbps, chunks, decode_gbps=5000.0, entry_bytes=12, decode_hidden=0.0):
    bw = link_gbps * 1e9 / 1e3   # bytes per ms
    L = int(rec["layout"].split("x")[0])
    q = int(rec["layout"].split("x")[1])
    # panels: q pieces of A along the grid row and q of B along the grid column arrive, the own ones do not move
    panel_bytes = (rec["nnz_A_panel"] + rec["nnz_B_panel"]) * entry_bytes * (q - 1) / q
    bcast = panel_bytes / bw
    ph = rec["phases_ms"]
    if rec.get("fiber_mode") == "gather":
        # the fiber gather: the partners swap their layer operands (both directions at once, one link), then one
        # product of the full inner dimension for the own column half; no codec, no merge
        xfer = max(rec.get("gather_bytes_sent", 0), rec.get("gather_bytes_recv", 0)) / bw
        compute = sum(p["total_ms"] for p in ph)
        return bcast + xfer + compute, {"bcast": bcast, "gather": xfer, "compute": compute, "encode": 0.0,
                                        "fiber_exposed": 0.0, "decode": 0.0, "merge": 0.0}
    if L == 1 or not rec.get("fiber"):
        compute = sum(p["total_ms"] for p in ph)
        return bcast + compute, {"bcast": bcast, "compute": compute, "encode": 0.0, "fiber_exposed": 0.0, "decode": 0.0,
                                 "merge": 0.0}
    codec = rec.get("fiber_codec") or {}
    enc = float(codec.get("encode_ms", 0.0))
    t_other, t_mine = ph[0]["total_ms"] + enc, ph[1]["total_ms"]
    wire = rec["fiber"]["bytes"]
    x = wire / chunks / bw
    send_end = 0.0
    for c in range(1, chunks + 1):
        send_end = max(c * t_other / chunks, send_end) + x
    compute_end = t_other + t_mine
    fiber_exposed = max(0.0, send_end - compute_end)
    # decode: the measured codec, else read the wire bytes and write the piece's rows and values at decode_gbps
    decode = float(codec["decode_ms"]) if "decode_ms" in codec else \
        (wire + rec.get("recv_nnz", 0) * entry_bytes) / (decode_gbps * 1e9 / 1e3)
    merge = rec["merge_ms"]
    # the pipeline decodes each chunk on a decode stream while the own half multiplies: the share of the decode the
    # overlap probe (tools/overlap_probe.py: product || codec on one GPU) measured as hidden leaves the step
    decode *= max(0.0, 1.0 - decode_hidden)
    total = bcast + compute_end + fiber_exposed + decode + merge
    return total, {"bcast": bcast, "compute": compute_end, "encode": enc, "fiber_exposed": fiber_exposed,
                   "decode": decode, "merge": merge}


def predict(records, link_gbps=64.0, chunks=2, decode_hidden=0.0):
    steps = [rank_step(r, link_gbps, chunks, decode_hidden=decode_hidden) for r in records]
    worst = max(range(len(steps)), key=lambda i: steps[i][0])
    mult = sum(r["multiplies"] for r in records)
    ms = steps[worst][0]
    return {"ranks": len(records), "layout": records[0]["layout"], "workload": records[0].get("config",
                                                                                              records[0].get("scale")),
            "link_GBps": link_gbps, "chunks": chunks, "step_ms": round(ms, 2),
            "multiplies": mult, "multiplies_per_s": mult / (ms / 1e3),
            "slowest_rank": records[worst]["rank"], "parts_ms": {k: round(v, 2) for k, v in steps[worst][1].items()}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("jsonl")
    ap.add_argument("--link-GBps", type=float, default=64.0)
    ap.add_argument("--link-from", default=None,
                    help="tools/p2p_probe.py output: its measured link_GBps replaces --link-GBps")
    ap.add_argument("--chunks", type=int, default=2)
    ap.add_argument("--decode-hidden", type=float, default=0.0,
                    help="share of the decode hidden behind the own-half product (tools/overlap_probe.py)")
    ap.add_argument("--overlap-from", default=None,
                    help="tools/overlap_probe.py output: the hidden share of the whole codec (hidden_frac_of_codec, "
                         "encode + decode overlapped together) as --decode-hidden -- conservative for the decode alone")
    a = ap.parse_args()
    if a.link_from:
        rec = json.load(open(a.link_from))
        if rec.get("link_GBps"):
            a.link_GBps = float(rec["link_GBps"])
    if a.overlap_from:
        o = json.loads([x for x in open(a.overlap_from) if x.startswith("{")][-1])
        a.decode_hidden = min(1.0, max(0.0, float(o["hidden_frac_of_codec"])))
    recs = [json.loads(l) for l in open(a.jsonl) if l.startswith("{")]
    groups = {}
    for r in recs:
        groups.setdefault((r.get("config", ""), r["layout"]), []).append(r)
    for g in groups.values():
        p = predict(g, a.link_GBps, a.chunks, a.decode_hidden)
        p["decode_hidden"] = round(a.decode_hidden, 3)
        print(json.dumps(p))


if __name__ == "__main__":
    main()
