"""Per-dispatch averages of rocprofv3 counter CSVs for one kernel:
    python profiles/pmc_sum.py <dir> <kernel-substring>"""
import collections
import csv
import glob
import sys

d, kname = sys.argv[1], sys.argv[2]
for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(float)
    disp = set()
    for r in csv.DictReader(open(f)):
        if kname not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
        disp.add(r["Dispatch_Id"])
    if disp:
        print(f, {k: round(v / len(disp)) for k, v in agg.items()}, "dispatches", len(disp))
for f in sorted(glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if kname in r["Name"]:
            print(f, r["Name"][:70], r["Calls"], r["AverageNs"])
