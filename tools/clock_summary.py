"""Summarise tools/clock_probe.sh: effective clock = GRBM_GUI_ACTIVE / 8 / duration for the
longest dispatches (the quotient reads high on dispatches shorter than ~0.3 ms), and the MFMA
pipe's busy cycles per CU-cycle (SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 · 256 CUs))."""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
per = defaultdict(dict)
for f in glob.glob(os.path.join(d, "pmc", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        try:
            key = (r.get("Dispatch_Id"), r.get("Kernel_Name", "")[:70])
            per[key]["dur"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
            per[key][r["Counter_Name"]] = per[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        except (KeyError, ValueError):
            continue
rows = sorted(((v["dur"], k[1], v) for k, v in per.items() if "dur" in v), key=lambda r: -r[0])
print("%10s %7s %9s %9s  %s" % ("dur_ms", "GHz", "mfma/cyc", "busy/cyc", "kernel"))
for dur, name, v in rows[:30]:
    g = v.get("GRBM_GUI_ACTIVE", float("nan"))
    cyc = g / 8.0
    print("%10.3f %7.3f %9.3f %9.3f  %s" % (dur * 1e-6, cyc / dur, v.get("SQ_VALU_MFMA_BUSY_CYCLES", float("nan")) / (cyc * 256),
                                       v.get("SQ_BUSY_CYCLES", float("nan")) / cyc, name))
