"""Read a traced persistent-factorisation launch (tools/dag_bench.cpp CSV) and print where the
time goes: per task type the wait (fetch -> inputs ready) and the run (ready -> outputs drained),
the leaf chain step by step (LEAF(k) -> TRSM(k+1,k) -> UPD(k+1,k+1,k) -> LEAF(k+1)), and the
hand-off latency (a consumer's ready time minus the done time of the last producer it waited on).
Usage: python tools/dag_trace.py trace.csv"""
import csv
import sys
from collections import defaultdict

NAMES = {0: "LEAF", 1: "TRSM", 2: "UPD", 3: "UPDX", 4: "FIN", 5: "LEAF'", 6: "INV", 7: "TRSM'"}
TICK_US = 0.01  # s_memrealtime runs at 100 MHz


def load(path):
    rows = []
    for r in csv.DictReader(open(path)):
        w = int(r["word"])
        rows.append(dict(slot=int(r["slot"]), type=w & 7, part=(w >> 3) & 15, fine=(w >> 7) & 1, i=(w >> 8) & 255,
                         j=(w >> 16) & 255, k=(w >> 24) & 255, fetch=int(r["fetch"]),
                         ready=int(r["ready"]), done=int(r["done"]), wg=int(r["wg"]),
                         xcc=int(r["xcc"])))
    t0 = min(r["fetch"] for r in rows)
    for r in rows:
        for key in ("fetch", "ready", "done"):
            r[key] = (r[key] - t0) * TICK_US
    return rows


def main():
    rows = load(sys.argv[1])
    span = max(r["done"] for r in rows)
    print(f"{len(rows)} slots, span {span:.1f} us")
    by = defaultdict(list)
    for r in rows:
        by[r["type"]].append(r)
    print(f"{'type':6s} {'n':>6s} {'wait us':>9s} {'run us':>9s} {'run p90':>9s}")
    for t in sorted(by):
        rs = by[t]
        run = sorted(r["done"] - r["ready"] for r in rs)
        wait = sum(r["ready"] - r["fetch"] for r in rs) / len(rs)
        print(f"{NAMES[t]:6s} {len(rs):6d} {wait:9.2f} {sum(run) / len(run):9.2f} {run[int(0.9 * (len(run) - 1))]:9.2f}")
    # tile-task completion = last strip done; readiness = first strip ready
    done, ready = {}, {}
    for r in rows:
        key = (r["type"], r["i"], r["j"], r["k"])
        done[key] = max(done.get(key, 0.0), r["done"])
        ready[key] = min(ready.get(key, 1e30), r["ready"])
    T = max(r["i"] for r in rows) + 1
    print("\nleaf chain: k, LEAF ready/run, ->TRSM(k+1,k) hand-off + run, ->UPD(k+1,k+1,k) hand-off + run, ->LEAF(k+1) hand-off")
    tot = defaultdict(float)
    for k in range(T):
        lt = 5 if (5, k, k, k) in done else 0
        lk = (lt, k, k, k)
        line = f"k={k:2d} leaf @{ready[lk]:8.1f} run {done[lk] - ready[lk]:6.1f}"
        tot["leaf"] += done[lk] - ready[lk]
        if k + 1 < T:
            tr = (7 if (7, k + 1, k, k) in done else 1, k + 1, k, k)
            up = (2, k + 1, k + 1, k)
            nl = (lt, k + 1, k + 1, k + 1)
            h1 = ready[tr] - done[lk]
            r1 = done[tr] - ready[tr]
            h2 = ready[up] - done[tr]
            r2 = done[up] - ready[up]
            h3 = ready[nl] - done[up]
            tot["h"] += h1 + h2 + h3
            tot["trsm"] += r1
            tot["upd"] += r2
            line += f" | trsm +{h1:5.1f} run {r1:5.1f} | upd +{h2:5.1f} run {r2:5.1f} | leaf +{h3:5.1f}"
        print(line)
    last_leaf = done[(5 if (5, T - 1, T - 1, T - 1) in done else 0, T - 1, T - 1, T - 1)]
    print(f"\nchain totals: leaves {tot['leaf']:.1f} us, TRSM runs {tot['trsm']:.1f}, UPD runs {tot['upd']:.1f}, "
          f"hand-offs {tot['h']:.1f}; last leaf done @{last_leaf:.1f}, tail (inverse) {span - last_leaf:.1f} us")
    busy = sum(r["done"] - r["ready"] for r in rows)
    wgs = len({r["wg"] for r in rows})
    print(f"work (sum of runs) {busy:.0f} us over {wgs} workgroups = {busy / (wgs * span):.1%} of the span")


if __name__ == "__main__":
    main()
