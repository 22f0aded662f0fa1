"""Mean per-dispatch counter values of one kernel from tools/pmc_*.sh output.
Usage: python tools/pmc_summary.py DIR [KERNEL_SUBSTRING]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "k_integrate<true, true, false, false, false, false, true>"
for f in sorted(glob.glob(f"{d}/[pe]*/run_counter_collection.csv")):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        print(f"{f.split('/')[-2]} {k:40s} n={len(v)} mean={sum(v) / len(v):.4g}")
