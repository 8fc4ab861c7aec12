"""Where one production C3 unit's time goes, per stream, from a rocprofv3 kernel trace:
the main stream's busy time by kernel class, the idle gaps before each class (what the main
stream waited on: launch boundaries, the side stream's join, the host), and the side stream.
Usage: python tools/critpath.py <run_kernel_trace.csv> [unit_index]
Units are delimited by the K_ff Gram launches (gram_mfma_kernel<8, true>, gram_reg_kernel<8> before round 5)."""
import csv
import sys
from collections import defaultdict


def cls(name, grid):
    n = name.split("(")[0].replace("void ", "").replace("gps::", "")
    if n.startswith("gemm_f64_kernel"):
        return "gemm128/64 " + n[len("gemm_f64_kernel"):]
    if n.startswith("gemm_f64_small_kernel") or n.startswith("gemm_f64_tiny_kernel"):
        return "gemm_small"
    return n


rows = []
for r in csv.DictReader(open(sys.argv[1])):
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                 int(r["Queue_Id"]), int(r["Queue_Id"]), int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"])))
rows.sort()
kff = [i for i, k in enumerate(rows) if ("gram_reg_kernel<8>" in k[2] or "gram_mfma_kernel<8" in k[2]) and k[5] > 5_000_000]
u = int(sys.argv[2]) if len(sys.argv) > 2 else 1
a = kff[u]
b = kff[u + 1] if u + 1 < len(kff) else len(rows)
win = rows[a:b]
t0, t1 = win[0][0], max(k[1] for k in win)
print("unit %d: %d dispatches, span %.3f ms" % (u, len(win), (t1 - t0) / 1e6))
streams = defaultdict(list)
for k in win:
    streams[k[3]].append(k)
main = max(streams, key=lambda s: len(streams[s]))
for s, ks in sorted(streams.items()):
    busy = sum(e - st for st, e, *_ in ks)
    print("queue %d%s: %d kernels, busy %.3f ms" % (s, " (main)" if s == main else "", len(ks), busy / 1e6))
ks = streams[main]
dur = defaultdict(float)
cnt = defaultdict(int)
gap_before = defaultdict(float)
prev_end = ks[0][0]
for st, e, nm, _, _, g in ks:
    c = cls(nm, g)
    dur[c] += e - st
    cnt[c] += 1
    gap_before[c] += max(0, st - prev_end)
    prev_end = max(prev_end, e)
tot_gap = sum(gap_before.values())
lv = sorted((e - st) / 1e3 for st, e, nm, *_ in ks if "potrf_diag" in nm)
if lv:
    print("leaves: %d, median %.1f us, sum %.3f ms, the 5 longest: %s" % (
        len(lv), lv[len(lv) // 2], sum(lv) / 1e3, " ".join("%.0f" % v for v in lv[-5:])))
print("main queue: busy %.3f ms, gaps %.3f ms" % (sum(dur.values()) / 1e6, tot_gap / 1e6))
print("%-34s %6s %10s %10s %9s" % ("class", "n", "busy ms", "gap ms", "avg us"))
for c in sorted(dur, key=lambda c: -(dur[c] + gap_before[c])):
    print("%-34s %6d %10.3f %10.3f %9.1f" % (c[:34], cnt[c], dur[c] / 1e6, gap_before[c] / 1e6,
                                             dur[c] / cnt[c] / 1e3))
