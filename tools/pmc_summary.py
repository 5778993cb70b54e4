#!/usr/bin/env python3
"""Summarise a tools/profile_gpu.sh output dir: per-kernel averages of every
collected counter + kernel-trace stats. Usage: pmc_summary.py <prof_dir> [kernel-substring]"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
ksub = sys.argv[2] if len(sys.argv) > 2 else "scan_dfa8"
out = []
st = os.path.join(d, "trace", "run_kernel_stats.csv")
if os.path.exists(st):
    for r in csv.DictReader(open(st)):
        out.append("trace  %-60s calls=%s avg_ns=%.0f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"])))
agg = collections.defaultdict(list)
for f in glob.glob(os.path.join(d, "pmc_*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if ksub in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(agg):
    v = agg[k]
    out.append("pmc    %-28s n=%d avg=%.6g" % (k, len(v), sum(v) / len(v)))
print("\n".join(out))
