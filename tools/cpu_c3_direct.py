"""One direct timing of the oracle's ref-mirror (the reference op sequence) at the full C3
size on the host cores, to check bench.py's cpu_baseline extrapolation (C2 × 64).
Prints a heartbeat every 30 s (the run takes minutes) and one JSON line at the end.
    python tools/cpu_c3_direct.py > gpurun_out/cpu_c3.json
"""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import bench  # noqa: E402
import gp_oracle as O  # noqa: E402


def main():
    done = threading.Event()
    t0 = time.perf_counter()

    def beat():
        while not done.wait(30):
            print(f"# ref_full C3 running {time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)

    threading.Thread(target=beat, daemon=True).start()
    out = {}
    for name in ("C2", "C3"):
        c = bench.CONFIGS[name]
        X, y, Xt, yt, _, th = bench.synth(c["n"], c["d"], c["nt"], c["seed"])
        t1 = time.perf_counter()
        O.ref_full(X, y, Xt, yt, *th)
        out[name] = time.perf_counter() - t1
    done.set()
    cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    print(json.dumps({"c2_s": out["C2"], "c3_s": out["C3"], "c2_x64_s": 64 * out["C2"],
                      "cores": cores, "kind": "port (oracle ref_full)"}))


if __name__ == "__main__":
    main()
