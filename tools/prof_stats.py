#!/usr/bin/env python3
"""Kernel statistics (rocprofv3 --kernel-trace --stats style CSV) from a rocprofv3 rocpd database.
usage: python tools/prof_stats.py run_results.db [out.csv]"""
import collections
import csv
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
rows = db.execute("select s.display_name, d.end - d.start from rocpd_kernel_dispatch d "
                  "join rocpd_info_kernel_symbol s on d.kernel_id = s.id").fetchall()
agg = collections.defaultdict(list)
for name, dur in rows:
    agg[name].append(dur)
tot = sum(sum(v) for v in agg.values())
out = [("Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs")]
for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    out.append((name, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / tot, min(v), max(v)))
w = csv.writer(open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout)
w.writerows(out)
