"""Summarise tools/gap_probe.sh: over the last C3 unit's dispatches (between the last two
gram_kernel launches of K_ff), busy time (union of kernel intervals) vs span, and the gap
distribution after short kernels."""
import csv
import glob
import os
import sys

d = sys.argv[1]
ks = []
for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
ks.sort()
grams = [i for i, k in enumerate(ks) if "gram_kernel" in k[2]]
# one unit = fit (gram K_ff ... ) + predict (gram K*f ...): take the last 4 gram launches' window
start = grams[-4] if len(grams) >= 4 else 0
win = ks[start:]
t0, t1 = win[0][0], max(k[1] for k in win)
busy, cur_s, cur_e = 0, None, None
for s, e, _ in win:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
print("dispatches %d  span %.3f ms  busy(union) %.3f ms  idle %.3f ms" % (len(win), (t1 - t0) * 1e-6, busy * 1e-6, (t1 - t0 - busy) * 1e-6))
gaps = []
for a, b in zip(win, win[1:]):
    g = b[0] - a[1]
    if g > 0:
        gaps.append((g, a[2][:40], a[1] - a[0]))
gaps.sort()
import statistics
gv = [g for g, _, _ in gaps]
if gv:
    print("positive gaps: n %d  median %.2f us  p90 %.2f us  sum %.3f ms" % (len(gv), statistics.median(gv) * 1e-3, gv[int(0.9 * len(gv))] * 1e-3, sum(gv) * 1e-6))
short = [(b[1] - b[0]) for b in win if b[1] - b[0] < 20000]
print("dispatches shorter than 20 us: %d, total %.3f ms" % (len(short), sum(short) * 1e-6))
