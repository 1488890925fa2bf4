"""Kernel stats and one product chain's timeline from a rocprofv3 results database (rocpd sqlite).

usage: python tools/db_timeline.py RESULTS.db FIRST_KERNEL_SUBSTRING [OCCURRENCE_FROM_END]
Prints a per-kernel summary (calls, total, average) and the dispatches and copies between the chosen
occurrence of FIRST_KERNEL_SUBSTRING and the next one, with the idle gap before each.
"""
import re
import sqlite3
import sys


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("cbg::", "").replace("void ", "")
    return re.sub(r"\(.*", "", n)[:70]


def main():
    db, first = sys.argv[1], sys.argv[2]
    back = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    c = sqlite3.connect(db)
    ks = list(c.execute("select name, start, end, grid_x from kernels order by start"))
    mc = list(c.execute("select start, end, size from memory_copies order by start"))
    agg = {}
    for n, s, e, _ in ks:
        a = agg.setdefault(short(n), [0, 0])
        a[0] += 1
        a[1] += e - s
    print("calls,total_us,avg_us,kernel")
    for n, (k, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
        print(f"{k},{t / 1e3:.1f},{t / 1e3 / k:.1f},{n}")
    idx = [i for i, k in enumerate(ks) if first in k[0]]
    i0, i1 = idx[-back], idx[-back + 1]
    t0 = ks[i0][1]
    ev = [(s, e, f"{short(n)} grid {g}") for n, s, e, g in ks[i0:i1]]
    ev += [(s, e, f"copy {z} B") for s, e, z in mc if t0 <= s < ks[i1][1]]
    ev.sort()
    print("\nstart_us,dur_us,gap_us,what")
    prev = t0
    for s, e, n in ev:
        print(f"{(s - t0) / 1e3:.1f},{(e - s) / 1e3:.1f},{(s - prev) / 1e3:.1f},{n}")
        prev = e
    print(f"span_us,{(ev[-1][1] - t0) / 1e3:.1f}")


if __name__ == "__main__":
    main()
