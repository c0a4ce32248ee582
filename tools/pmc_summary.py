#!/usr/bin/env python3
"""Mean of every PMC counter per kernel over the dispatches of rocprofv3 --pmc runs.
Usage: pmc_summary.py <dir-glob> [kernel-substring]"""
import collections
import csv
import glob
import re
import sys

pat = sys.argv[1]
ksub = sys.argv[2] if len(sys.argv) > 2 else "k_spmv"
agg = collections.defaultdict(list)
for f in sorted(glob.glob(pat + "/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if ksub in r["Kernel_Name"]:
            k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void spmvhw::", "")
            agg[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    print(f"{k:60s} {c:36s} n={len(v):3d} mean={sum(v) / len(v):.6g}")
