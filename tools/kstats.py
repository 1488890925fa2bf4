#!/usr/bin/env python3
"""Short table of a rocprofv3 *kernel_stats.csv: kernel (template args kept), calls, avg ms."""
import csv
import sys

for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    k = n.find("k_")
    n = n[k:n.find("(", k)] if k >= 0 else n[:40]
    print(f"{n:60s} {r['Calls']:>4} {float(r['AverageNs']) / 1e6:8.3f} ms")
