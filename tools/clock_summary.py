"""Summarise tools/clock_probe.sh: effective clock = GRBM_GUI_ACTIVE / 8 / duration for the
longest dispatches (the quotient reads high on dispatches shorter than ~0.3 ms)."""
import csv
import glob
import os
import sys

d = sys.argv[1]
rows = []
for f in glob.glob(os.path.join(d, "pmc", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        try:
            val = float(r.get("Counter_Value", "nan"))
            t0, t1 = float(r.get("Start_Timestamp", "nan")), float(r.get("End_Timestamp", "nan"))
        except ValueError:
            continue
        rows.append((t1 - t0, val, name[:70]))
rows.sort(reverse=True)
print("%10s %8s  %s" % ("dur_ms", "GHz", "kernel"))
for dur, val, name in rows[:25]:
    if dur > 0:
        print("%10.3f %8.3f  %s" % (dur * 1e-6, val / 8 / dur, name))
