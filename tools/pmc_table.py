"""Per-kernel averages of rocprofv3 --pmc counter_collection.csv files.
usage: python tools/pmc_table.py <dir> [<dir> ...]"""
import collections
import csv
import glob
import os
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        names = {}
        for r in csv.DictReader(open(f)):
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        for did, cs in per.items():
            for c, v in cs.items():
                agg[names[did]][c].append(v)
cols = sorted({c for cs in agg.values() for c in cs})
print("kernel," + ",".join(cols))
for k, cs in agg.items():
    print(k[:48] + "," + ",".join(f"{sum(cs[c]) / len(cs[c]):.4g}" if cs.get(c) else "" for c in cols))
