"""Sum a rocprofv3 counter_collection.csv per kernel and counter, per launch.
    python tools/pmc_dump.py <dir> [kernel-substring ...]"""
import collections
import csv
import glob
import sys

files = glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True)
want = sys.argv[2:]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in files:
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if want and not any(w in k for w in want):
            continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
for k, v in acc.items():
    n = max(1, len(disp[k]))
    print(k[-60:], n, {c: round(x / n) for c, x in sorted(v.items())})
