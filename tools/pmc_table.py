#!/usr/bin/env python3
"""Mean per-dispatch counter values of the rx kernels (or the kernels whose name
contains argv[2]) from pmc_probe.sh / slice_pmc.sh output dirs."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
name = sys.argv[2] if len(sys.argv) > 2 else "rx_"
rows = collections.defaultdict(dict)
for d in sorted(glob.glob(os.path.join(root, "k*_*"))):
    if not os.path.isdir(d):
        continue
    kind = os.path.basename(d).split("_")[0]
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if name in r["Kernel_Name"]:
                acc[(r["Counter_Name"], r["Dispatch_Id"])].append(float(r["Counter_Value"]))
    per = collections.defaultdict(list)
    for (c, _), v in acc.items():
        per[c].append(sum(v))
    for c, v in per.items():
        rows[c][kind] = sum(v) / len(v)
kinds = sorted({k for r in rows.values() for k in r})
print("counter".ljust(30) + "".join(k.rjust(16) for k in kinds))
for c in sorted(rows):
    print(c.ljust(30) + "".join(f"{rows[c].get(k, float('nan')):16.4g}" for k in kinds))
