"""Summarise rocprofv3 --pmc CSVs: per-dispatch counter values of rc1pass_kernel,
averaged over its dispatches.  Usage: python tools/pmc_summary.py gpurun_out/pmc"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "rc1pass_kernel"
# optional: only dispatches of this grid size (e.g. the steady-state frames that
# run the learned launch order: their grid is the order's slot count)
grid = os.environ.get("PMC_GRID")
vals = defaultdict(list)
durations = []
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    per = defaultdict(float)
    with open(f) as fh:
        for row in csv.DictReader(fh):
            if kern not in row.get("Kernel_Name", ""):
                continue
            if grid and str(row.get("Grid_Size", "")) != grid:
                continue
            per[(row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
    for (d, name), v in per.items():
        vals[name].append(v)
for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            if kern in row.get("Kernel_Name", "") and (not grid or str(row.get("Grid_Size_X", row.get("Grid_Size", ""))) == grid):
                durations.append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
out = {k: sum(v) / len(v) for k, v in sorted(vals.items())}
out["_dispatches_per_counter"] = {k: len(v) for k, v in sorted(vals.items())}
if durations:
    out["_kernel_ns_avg"] = sum(durations) / len(durations)
print(json.dumps(out, indent=1))
