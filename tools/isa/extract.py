#!/usr/bin/env python3
"""dev helper: print one kernel's body from a hipcc -S file.  usage: extract.py file.s substring"""
import sys
lines = open(sys.argv[1]).read().split("\n")
st = next(i for i, l in enumerate(lines) if sys.argv[2] in l and l.rstrip().endswith(":") is False and l.startswith("_Z") and ":" in l)
en = next(i for i in range(st, len(lines)) if lines[i].startswith(".Lfunc_end"))
print("\n".join(lines[st:en]))
