#!/usr/bin/env python3
"""Summarize tools/fq_counters.sh output: per kernel (substring) mean counter value per
dispatch. Usage: python3 tools/fq_pmc_summary.py TAG [kernel_substring ...]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

tag = sys.argv[1]
subs = sys.argv[2:] or ["k_fq_format", "k_fq_off", "k_fq_bsum"]
res = defaultdict(dict)
for d in sorted(glob.glob(f"gpurun_out/fqpmc_{tag}_*")):
    if not os.path.isdir(d):
        continue
    counter = d.split(f"fqpmc_{tag}_", 1)[1]
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        vals = defaultdict(list)
        for row in csv.DictReader(open(f)):
            name = row.get("Kernel_Name", "")
            for s in subs:
                if s in name:
                    vals[s].append(float(row["Counter_Value"]))
        for s, v in vals.items():
            # rows are per dispatch (and possibly per dimension); sum per dispatch is not
            # recoverable here, report the mean row value and the row count
            res[s][counter] = {"mean": sum(v) / len(v), "rows": len(v)}
print(json.dumps(res, indent=1))
