"""Per-launch averages of the counters tools/probe/pmc_ab.sh collected, per build."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
for d in sorted(glob.glob(os.path.join(root, "*"))):
    if not os.path.isdir(d):
        continue
    tot = defaultdict(float)
    n = defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "raster_kernel" not in r["Kernel_Name"]:
                continue
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            n[r["Counter_Name"]].add(r["Dispatch_Id"])
    print(os.path.basename(d), " ".join("%s=%.4g" % (k, tot[k] / max(len(n[k]), 1)) for k in sorted(tot)))
