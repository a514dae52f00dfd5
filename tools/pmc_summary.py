#!/usr/bin/env python3
"""Per-kernel mean of every PMC counter found under a rocprofv3 output tree."""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        per[(r["Kernel_Name"].split("(")[0], r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (k, _, c), v in per.items():
        acc[k][c].append(v)
out = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in acc.items()}
json.dump(out, open(os.path.join(root, "summary.json"), "w"), indent=1)
for k, d in out.items():
    if "xrt" not in k:
        continue
    print(k)
    for c in sorted(d):
        print("   %-28s %.4g" % (c, d[c]))
