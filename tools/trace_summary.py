#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 kernel_trace.csv, grouped by (name, grid):
calls, mean us, total ms, share.  Usage: python tools/trace_summary.py TRACE.csv [--top N]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 40
d = defaultdict(list)
for x in rows:
    key = (x["Kernel_Name"][:100], f'{x["Grid_Size_X"]}x{x["Grid_Size_Y"]}/{x["Workgroup_Size_X"]}')
    d[key].append((int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3)
tot = sum(sum(v) for v in d.values())
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:top]:
    print(f"{len(v):5d} {sum(v)/len(v):10.1f}us {sum(v)/1e3:9.2f}ms {100*sum(v)/tot:5.1f}%  {k[1]:>18}  {k[0]}")
print(f"total {tot/1e3:.2f} ms")
