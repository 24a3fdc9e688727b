"""Summarise rocprofv3 --pmc CSVs: mean per dispatch of each counter for one kernel.
    python tools/pmc_summary.py gpurun_out/pmc_TAG [kernel-substring]"""
import csv, glob, json, os, sys
from collections import defaultdict
d = sys.argv[1]; pat = sys.argv[2] if len(sys.argv) > 2 else "crc32c_fixed_kernel"
vals = defaultdict(lambda: defaultdict(float))
for f in sorted(glob.glob(os.path.join(d, "*counter_collection.csv"))):
    for row in csv.DictReader(open(f)):
        if pat not in row.get("Kernel_Name", ""):
            continue
        key = (f, row["Dispatch_Id"])
        vals[row["Counter_Name"]][key] += float(row["Counter_Value"])
out = {}
for c, per in vals.items():
    v = list(per.values())
    out[c] = sum(v) / len(v)
print(json.dumps({k: round(v, 1) for k, v in sorted(out.items())}, indent=1))
