"""Per-launch durations of the persistent factorisation in C3 units from a rocprofv3 kernel trace
(a rocprofv3 --kernel-trace of the C3 unit): the last unit's 8 launches, and whether a side-stream GEMM overlapped."""
import csv
import sys

for d in sys.argv[1:]:
    rows = list(csv.DictReader(open(d + "/run_kernel_trace.csv")))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dag = [r for r in rows if "potrf_dag_kernel" in r["Kernel_Name"]]
    last = dag[-8:]
    out = []
    for r in last:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        ov = [x for x in rows if x is not r and x["Queue_Id"] != r["Queue_Id"] and
              int(x["Start_Timestamp"]) < e and int(x["End_Timestamp"]) > s and
              "gemm" in x["Kernel_Name"]]
        out.append("%.0f%s" % ((e - s) / 1e3, "*" if ov else ""))
    tot = sum(float(x.rstrip("*")) for x in out)
    print("%-40s dag us: %s  sum %.0f  (* = a GEMM on another queue overlapped)" % (d, " ".join(out), tot))
