"""Dump one unit's kernels (start, end relative to the unit start, queue) from a rocprofv3
kernel trace, to read overlaps by eye.
Usage: python tools/timeline_dump.py <run_kernel_trace.csv> <first-kernel-substring> [unit]"""
import csv
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "").replace("gps::", ""), r["Queue_Id"]))
rows.sort()
marks = [i for i, k in enumerate(rows) if sys.argv[2] in k[2]]
u = int(sys.argv[3]) if len(sys.argv) > 3 else 1
a = marks[u]
b = marks[u + 1] if u + 1 < len(marks) else len(rows)
t0 = rows[a][0]
for s, e, n, q in rows[a:b]:
    print("%9.1f %9.1f %8.1f q%s %s" % ((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3, q, n[:60]))
