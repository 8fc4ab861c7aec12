"""Per-kernel L2-to-fabric traffic from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE csv passes.

FETCH_SIZE / WRITE_SIZE count the L2's memory-side (fabric) requests, Infinity-Cache (MALL)
hits included (MI355X_MICROARCH.md §HBM), so these are L2-miss bytes, an upper bound on
HBM bytes — not HBM bytes.  gfx950 correction: FETCH_SIZE reports half the bytes of a wide
coalesced streaming read, so read bytes = 2·FETCH_SIZE·1024; WRITE_SIZE is exact for
16-byte-per-lane streaming stores: write bytes = WRITE_SIZE·1024.
Writes <dir>/<sub>traffic.json with per-kernel-name averages per launch.
Usage: python tools/traffic.py gpurun_out/prof_<tag> [sub-prefix, e.g. "fitc_"]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(pattern):
    per = defaultdict(list)
    for f in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name") or r.get("Kernel-Name") or r.get("KernelName")
            val = r.get("Counter_Value") or r.get("Counter-Value")
            if name is None or val is None:
                continue
            per[name].append(float(val))
    return per


def short(name):
    name = name.replace("void ", "")
    return name[: name.find("(")] if "(" in name else name


def main(d, sub=""):
    fetch = load(os.path.join(d, sub + "fetch", "**", "*counter_collection.csv"))
    write = load(os.path.join(d, sub + "write", "**", "*counter_collection.csv"))
    out = {}
    for name in sorted(set(fetch) | set(write)):
        f, w = fetch.get(name, []), write.get(name, [])
        n = max(len(f), len(w))
        rd = 2.0 * 1024.0 * sum(f) / max(len(f), 1)
        wr = 1024.0 * sum(w) / max(len(w), 1)
        out[short(name)] = out.get(short(name), [])
        out[short(name)].append({"launches": n, "read_bytes_per_launch": rd,
                                 "write_bytes_per_launch": wr,
                                 "fabric_bytes_per_launch": rd + wr})
    # merge instantiations with the same short name (keep the per-instantiation list)
    summary = {}
    for k, lst in out.items():
        tot_l = sum(x["launches"] for x in lst)
        summary[k] = {"launches": tot_l,
                      "fabric_bytes_per_launch": sum(x["fabric_bytes_per_launch"] * x["launches"]
                                                  for x in lst) / max(tot_l, 1),
                      "instantiations": lst}
    # per-launch averages the bench's roofline objects quote (full-GP-only counter run:
    # the bench step runs its timed passes once each in the counter run)
    def avg(*prefixes):
        ks = [k for k in summary if k.startswith(prefixes)]
        n = sum(summary[k]["launches"] for k in ks)
        b = sum(summary[k]["fabric_bytes_per_launch"] * summary[k]["launches"] for k in ks)
        return b / n if n else None
    # (the persistent factorisation's launches carry the bottom blocks' MFMA work, so they are
    # part of the roofline's launch set, bench.roofline_mfma)
    summary["_roofline"] = {"gemm_per_launch_bytes": avg("gps::gemm_f64_kernel", "gps::gemm_f64_small_kernel",
                                                         "gps::dag::potrf_dag_kernel"),
                            "gram_per_launch_bytes": avg("gps::gram_kernel", "gps::gram_reg_kernel", "gps::gram_mfma_kernel"),
                            "kind": "L2-fabric bytes (TCC FETCH_SIZE + WRITE_SIZE: every L2 miss, "
                                    "Infinity-Cache hits included) — an upper bound on HBM bytes",
                            "note": "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE "
                                    "half-count correction), per launch"}
    json.dump(summary, open(os.path.join(d, sub + "traffic.json"), "w"), indent=1)
    for k, v in sorted(((k, v) for k, v in summary.items() if not k.startswith("_")),
                       key=lambda kv: -kv[1]["fabric_bytes_per_launch"] * kv[1]["launches"]):
        print(f"{k:60s} launches={v['launches']:6d}  fabric/launch={v['fabric_bytes_per_launch']/1e6:10.2f} MB")


    print(json.dumps(summary["_roofline"]))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
