"""Average per-dispatch PMC counter values of one kernel over rocprofv3 --pmc pass directories.
usage: python tools/pmc_dump.py gpurun_out/pmca KERNEL_SUBSTRING"""
import csv
import glob
import sys
from collections import defaultdict

prefix, kern = sys.argv[1], sys.argv[2]
vals = defaultdict(lambda: defaultdict(float))
for path in glob.glob(prefix + "*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(path)):
        if kern not in r.get("Kernel_Name", ""):
            continue
        vals[r["Counter_Name"]][(path, r.get("Dispatch_Id"))] += float(r["Counter_Value"])
for name in sorted(vals):
    v = list(vals[name].values())
    print(f"{name:28s} {sum(v) / len(v):16.4g}   (n={len(v)})")
