#!/usr/bin/env python3
"""Average PMC values per kernel from rocprofv3 counter CSVs: pmc_table.py DIR [DIR...]"""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    for p in sorted(glob.glob(d + "/**/*counter_collection.csv", recursive=True)):
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(p)):
            n = r["Kernel_Name"]
            for k in ("k_run", "k_classify", "k_step"):
                if k in n:
                    agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        print(p)
        for k, dd in agg.items():
            print("  ", k, " ".join("%s=%.3g" % (c, sum(v) / len(v)) for c, v in sorted(dd.items())))
