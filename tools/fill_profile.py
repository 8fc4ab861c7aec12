"""Chip-fill profile of one unit from a rocprofv3 kernel trace: at every instant, the
workgroups of the running kernels (summed over queues) against the 512 slots of two
workgroups per CU.  Reports the fill-weighted time, the time spent below half fill and
the kernels running then — where the latency-bound chain leaves the chip idle.
Usage: python tools/fill_profile.py <run_kernel_trace.csv> <first-kernel-substring> [unit] [stride]
(stride: marker kernels per unit, e.g. 2 Gram launches per full-GP unit, 3 per FITC unit)"""
import collections
import csv
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    wg = 1
    for ax in "XYZ":
        g = int(r.get("Grid_Size_" + ax, 1) or 1)
        w = int(r.get("Workgroup_Size_" + ax, 1) or 1)
        wg *= max(1, (g + w - 1) // w)
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("gps::", "")
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, wg))
rows.sort()
marks = [i for i, k in enumerate(rows) if sys.argv[2] in k[2]]
u = int(sys.argv[3]) if len(sys.argv) > 3 else 1
st = int(sys.argv[4]) if len(sys.argv) > 4 else 1
a = marks[u * st]
b = marks[(u + 1) * st] if (u + 1) * st < len(marks) else len(rows)
unit = rows[a:b]
t0 = unit[0][0]
t1 = max(e for _, e, _, _ in unit)
ev = sorted({t for s, e, _, _ in unit for t in (s, e)})
SLOTS = 512
fill_t = 0.0
low_t = 0.0
low_by = collections.Counter()
for lo, hi in zip(ev, ev[1:]):
    run = [(n, w) for s, e, n, w in unit if s <= lo and e >= hi]
    f = min(1.0, sum(w for _, w in run) / SLOTS)
    fill_t += f * (hi - lo)
    if f < 0.5:
        low_t += hi - lo
        key = " + ".join(sorted({n[:40] for n, _ in run})) or "(nothing)"
        low_by[key] += hi - lo
span = (t1 - t0) / 1e6
print("unit %d: span %.3f ms, fill-weighted %.3f ms (%.1f %%), below half fill %.3f ms"
      % (u, span, fill_t / 1e6, 100 * fill_t / (t1 - t0), low_t / 1e6))
for k, v in low_by.most_common(12):
    print("  %8.3f ms  %s" % (v / 1e6, k))
