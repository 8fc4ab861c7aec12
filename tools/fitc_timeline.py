"""One FITC C4 unit's kernels on the timeline (the second of tools/fitc_unit.py's two units)
from a rocprofv3 --kernel-trace CSV: start / end / duration per kernel with its queue, and per
queue the busy time, so the critical path and what overlaps it can be read off.
Usage: python tools/fitc_timeline.py <kernel_trace.csv> [unit=1]"""
import csv
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), q, r["Kernel_Name"]))
rows.sort()
# units start at the K(Z,Z) Gram: the first gram launch after a gap of > 1 ms, or every
# gram_kmm-sized Gram; take the Gram launches of the m x m block by their short duration
starts = [i for i, k in enumerate(rows) if "gram" in k[3] and (i == 0 or k[0] - rows[i - 1][1] > 1_000_000)]
u = int(sys.argv[2]) if len(sys.argv) > 2 else 1
a = starts[u] if u < len(starts) else starts[-1]
b = starts[u + 1] if u + 1 < len(starts) else len(rows)
win = rows[a:b]
t0 = win[0][0]
busy = {}
for s, e, q, name in win:
    short = name.split("(")[0].replace("gps::", "")[:60]
    print(f"{(s - t0) / 1e3:10.1f} {(e - t0) / 1e3:10.1f} {(e - s) / 1e3:9.1f}  q{q}  {short}")
    busy[q] = busy.get(q, 0) + (e - s)
span = max(e for _, e, _, _ in win) - t0
print(f"span {span / 1e3:.1f} us; busy per queue: " + ", ".join(f"q{q} {v / 1e3:.1f}" for q, v in busy.items()))
