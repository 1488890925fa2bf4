#!/usr/bin/env python3
"""Per-kernel summary of rocprofv3 PMC passes (counter_collection.csv files) -> JSON.

    python tools/pmc_summary.py <out.json> <pass_dir> [<pass_dir> ...]

For every kernel (name truncated at the template arguments) and counter: the mean over dispatches of
the per-dispatch value (a dispatch's rows are summed over dimensions/instances).  Derived figures for
each kernel, where its counters are present:
  * wait / issue / active fractions of SQ_WAVE_CYCLES (SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY);
  * LDS-issue stall share (SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES), bank conflict cycles per LDS instruction;
  * HBM bytes = FETCH_SIZE + WRITE_SIZE (KiB x 1024) and the guide's doubled-FETCH upper bound
    (MI355X_MICROARCH.md, HBM: FETCH_SIZE reads 1/2 of a 16-B/lane streaming read on gfx950).
"""
import csv
import glob
import json
import os
import sys


def short(name):
    n = name.split("(")[0]
    for tag in ("k_num_heavy", "k_sym_part", "k_num_block", "k_num_wave", "k_sym_block", "k_sym_wave",
                "k_window", "k_col_stats", "k_unit_segs", "k_split_fill", "k_bin", "k_scan"):
        if tag in name:
            # keep the template arguments that distinguish instantiations (table size etc.)
            i = name.find(tag)
            j = name.find("(", i)
            return name[i:j if j > 0 else None][:120]
    return n[:120]


def load(dirs):
    per = {}   # (kernel, dispatch, counter) -> value
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                key = (short(r["Kernel_Name"]), d + ":" + r["Dispatch_Id"], r["Counter_Name"])
                per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
    agg = {}
    for (k, disp, c), v in per.items():
        agg.setdefault(k, {}).setdefault(c, []).append(v)
    out = {}
    for k, cs in agg.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        m["_dispatches"] = max(len(v) for v in cs.values())
        d = {}
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in m:
                    d[c + "/WAVE_CYCLES"] = m[c] / wc
        if m.get("SQ_INSTS_LDS") and "SQ_LDS_BANK_CONFLICT" in m:
            d["LDS_BANK_CONFLICT_per_LDS_inst"] = m["SQ_LDS_BANK_CONFLICT"] / m["SQ_INSTS_LDS"]
        if "FETCH_SIZE" in m:
            d["fetch_bytes"] = m["FETCH_SIZE"] * 1024.0
        if "WRITE_SIZE" in m:
            d["write_bytes"] = m["WRITE_SIZE"] * 1024.0
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            d["hbm_bytes"] = d["fetch_bytes"] + d["write_bytes"]
            d["hbm_bytes_fetch_doubled"] = 2 * d["fetch_bytes"] + d["write_bytes"]
        if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m and (m["TCC_HIT_sum"] + m["TCC_MISS_sum"]) > 0:
            d["L2_hit_rate"] = m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
        out[k] = {"counters": m, "derived": d}
    return out


def main():
    if len(sys.argv) < 3:
        sys.exit(__doc__)
    res = load(sys.argv[2:])
    json.dump(res, open(sys.argv[1], "w"), indent=1, sort_keys=True)
    for k in sorted(res, key=lambda k: -res[k]["counters"].get("SQ_WAVE_CYCLES", 0)):
        print(k, json.dumps(res[k]["derived"]))


if __name__ == "__main__":
    main()
