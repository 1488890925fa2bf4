#!/usr/bin/env python3
"""The fiber wire codec (cbg_fiber_codec: grid.hip's fiber_encode + fiber_decode) on the 1x1x2 layout's message at
full size on one GPU: rank 0's product of the other layer's columns, P = A[:, K_0] * A[K_0, J_1] with K_0 = the
first half of the inner dimension and J_1 the second half of the columns (cbg_rmat_block pieces).  Prints encode /
decode ms (HIP events), wire bytes per entry and the round-trip verdict; run it under rocprofv3 for the kernels.
usage: python tools/bench_codec.py [--scale S] [--chunks C] [--reps R]"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=21)
    ap.add_argument("--chunks", type=int, default=2)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import combblas_amd as cb
    ctx = cb.Context(0)
    n = 1 << a.scale
    h = n // 2
    Ak = ctx.rmat_block(a.scale, 0, n, 0, h)
    Bk = ctx.rmat_block(a.scale, 0, h, h, n)
    P = cb.LocalSpGEMMHash(cb.PlusTimesSRing("f64"), Ak, Bk)
    Ak.free()
    Bk.free()
    recs = [P.fiber_codec(a.chunks) for _ in range(a.reps + 1)][1:]
    best = min(recs, key=lambda r: r["encode_ms"] + r["decode_ms"])
    n_e = best["entries"]
    gb_enc = n_e * 12 * 2 / 1e9 + best["wire_bytes"] / 1e9          # two reads of rows + values, the stream written
    gb_dec = best["wire_bytes"] / 1e9 + n_e * 12 / 1e9              # the stream read, rows + values written
    print(json.dumps({"scale": a.scale, "chunks": a.chunks, "entries": n_e, "columns": best["columns"],
                      "wire_bytes": best["wire_bytes"], "bytes_per_entry": round(best["wire_bytes"] / n_e, 3),
                      "row_formats": best["row_formats"], "value_formats": best["value_formats"],
                      "roundtrip_exact": all(r["roundtrip_exact"] for r in recs),
                      "encode_ms": [round(r["encode_ms"], 3) for r in recs],
                      "decode_ms": [round(r["decode_ms"], 3) for r in recs],
                      "encode_GBps": round(gb_enc / (best["encode_ms"] / 1e3), 1),
                      "decode_GBps": round(gb_dec / (best["decode_ms"] / 1e3), 1)}), flush=True)


if __name__ == "__main__":
    main()
