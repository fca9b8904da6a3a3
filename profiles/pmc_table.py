"""Print per-kernel averages of every counter in a counters.sh output dir."""
import csv
import glob
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(sys.argv[1] + "/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("void ", "").replace("nrms::(anonymous namespace)::", "").split("(")[0]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    if "nrms" not in k and "kernel" not in k:
        continue
    print(k)
    for c in sorted(cs):
        v = cs[c]
        print(f"  {c:32s} {sum(v) / len(v):16.1f}  (n={len(v)})")
