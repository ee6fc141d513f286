"""Print the last training step's kernel timeline from a rocprofv3 kernel-trace
CSV (the launches between the last two adamw launches): start offset, duration
grid size and hardware queue per kernel.  Usage: step_timeline.py TRACE.csv"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
a, b = idx[-2] + 1, idx[-1] + 1
t0 = int(rows[a]["Start_Timestamp"])
queues = {}
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    q = queues.setdefault(r.get("Queue_Id", "?"), f"q{len(queues) + 1}")
    print(f'{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} {r["Grid_Size_X"]:>8} {q} {r["Kernel_Name"][:80]}')
print(f'step span {(int(rows[b - 1]["End_Timestamp"]) - t0) / 1e3:.1f} us')
