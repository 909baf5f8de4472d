"""Per-dispatch means of rocprofv3 --pmc counters for the kernels whose name contains a pattern.
Usage: pmc_summary.py <rocprofv3 output dir> <kernel substring> -> one JSON line."""
import csv
import glob
import json
import sys
from collections import defaultdict

d, pat = sys.argv[1], sys.argv[2]
files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
vals = defaultdict(lambda: defaultdict(float))
for f in files:
    with open(f, newline="") as fh:
        for row in csv.DictReader(fh):
            if pat not in row.get("Kernel_Name", ""):
                continue
            vals[row["Counter_Name"]][row.get("Dispatch_Id", "0")] += float(row["Counter_Value"])
out = {"kernel": pat, "files": len(files)}
for c, per in sorted(vals.items()):
    out[c] = round(sum(per.values()) / max(1, len(per)), 1)
    out["dispatches"] = len(per)
print(json.dumps(out))
