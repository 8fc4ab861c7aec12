"""Idle-time anatomy of one full-GP unit from a rocprofv3 kernel trace: the window from
one K_ff gram launch to the next, busy (union of kernel intervals) vs span, and the
idle time bucketed by what ran just before the gap.
Usage: python tools/unit_timeline.py <run_kernel_trace.csv> [unit_index]"""
import csv
import sys
from collections import defaultdict

ks = []
for r in csv.DictReader(open(sys.argv[1])):
    ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
ks.sort()
kff = [i for i, k in enumerate(ks) if ("gram_kernel<8>" in k[2] or "gram_reg_kernel<8>" in k[2] or "gram_mfma_kernel<8" in k[2]) and k[1] - k[0] > 300000]
u = int(sys.argv[2]) if len(sys.argv) > 2 else 1
a, b = kff[u], kff[u + 1]
win = ks[a:b]
t0 = win[0][0]
t1 = max(k[1] for k in win)
busy, cs, ce = 0, None, None
idle_after = defaultdict(float)
last_name = None
for s, e, nme in win:
    if ce is None or s > ce:
        if ce is not None:
            busy += ce - cs
            idle_after[last_name] += s - ce
        cs, ce = s, e
    else:
        ce = max(ce, e)
    if e >= ce:
        last_name = nme.split("(")[0].replace("void ", "")
busy += ce - cs
print("dispatches %d span %.3f ms busy %.3f ms idle %.3f ms" % (len(win), (t1 - t0) / 1e6,
                                                             busy / 1e6, (t1 - t0 - busy) / 1e6))
for k, v in sorted(idle_after.items(), key=lambda kv: -kv[1])[:10]:
    print("  idle after %-55s %.3f ms" % (k[:55], v / 1e6))
# time where only "small" kernels run (< 100 us): latency-bound phases
small = sum(e - s for s, e, _ in win if e - s < 100000)
print("kernel time in launches < 100 us: %.3f ms (sum of durations)" % (small / 1e6))
