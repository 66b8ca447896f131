#!/usr/bin/env python3
"""Per-dispatch mean of rocprofv3 --pmc counters for the env kernels, from
gpurun_out/<dir>/run_counter_collection.csv passes: pmc_compare.py <tag>..."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for tag in sys.argv[1:]:
    agg = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(root, "gpurun_out", f"pmc_{tag}_*", "**", "*counter_collection.csv"),
                              recursive=True)):
        for r in csv.DictReader(open(f)):
            if "env_kernel" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f"== {tag}")
    for k in sorted(agg):
        v = agg[k]
        print(f"  {k:24s} {sum(v) / len(v):16.1f}  (n={len(v)})")
