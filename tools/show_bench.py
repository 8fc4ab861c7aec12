"""Pretty-print a bench.py JSON line (tools/show_bench.py gpurun_out/bench.json)."""
import json
import sys

r = json.load(open(sys.argv[1]))
print("value %.4f %s | ms/step %.2f" % (r["value"], r["unit"], r["ms_per_step"]))
for k in ("roofline", "roofline_gram", "cpu_baseline"):
    if k in r:
        print(k, json.dumps({a: b for a, b in r[k].items() if a != "sample"}))
if "speedup_vs_cpu" in r:
    print("speedup_vs_cpu %.1f" % r["speedup_vs_cpu"])


def kern(d, ind="  "):
    for k, v in sorted(d.items(), key=lambda kv: -kv[1]["ms"]):
        extra = ("%.1f TF" % v["tflops"]) if v.get("tflops") else (("%.0f GB/s" % v["gbs"]) if v.get("gbs") else "")
        print("%s%-22s n=%6.1f  %9.3f ms  %s" % (ind, k, v["count"], v["ms"], extra))


kern(r["kernels_per_step"])
for obj, g in r.get("grad", {}).items():
    if isinstance(g, dict):
        print("GRAD %-9s %.2f ms/iteration  %.1f TF" % (obj, g["ms_per_iteration"], g["tflops"]))
for leg, f in r.get("fitc", {}).items():
    print("FITC %s: %.2f ms/step  gemm %.1f TF" % (leg, f["ms_per_step"], f["roofline"]["achieved"]))
    kern(f["kernels_per_step"], "    ")
