"""Sum / mean of rocprofv3 --pmc counters per kernel name from a counter_collection.csv
usage: python tools/exp/pmc_by_kernel.py DIR [name-substring]"""
import csv, glob, sys
from collections import defaultdict
rows = []
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
pat = sys.argv[2] if len(sys.argv) > 2 else ""
acc = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for r in rows:
    k = r["Kernel_Name"]
    if pat not in k:
        continue
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r["Dispatch_Id"])
for k, c in acc.items():
    n = len(disp[k])
    print(k[:90], "dispatches", n, {name: round(v / n) for name, v in sorted(c.items())})
