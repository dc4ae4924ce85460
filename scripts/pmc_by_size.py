#!/usr/bin/env python3
"""Per-dispatch FETCH_SIZE / WRITE_SIZE of one kernel from a scripts/profile_cmd.sh directory,
grouped by grid size (one row per problem size): mean KB per dispatch, and the traffic estimate
FETCH_SIZE x 2 + WRITE_SIZE (gfx950: FETCH_SIZE counts half of wide streaming reads,
MI355X_MICROARCH.md HBM section) in bytes.
usage: scripts/pmc_by_size.py DIR KERNEL_SUBSTRING"""
import collections
import csv
import glob
import json
import sys

d, kn = sys.argv[1], sys.argv[2]
res = collections.defaultdict(dict)
for part, ctr in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
    f = glob.glob(f"{d}/{part}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if kn not in r["Kernel_Name"] or r["Counter_Name"] != ctr:
            continue
        acc[r["Grid_Size"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for g, disp in acc.items():
        res[g][ctr + "_KB"] = sum(disp.values()) / len(disp)
        res[g]["dispatches_" + part] = len(disp)
for g, v in res.items():
    if "FETCH_SIZE_KB" in v and "WRITE_SIZE_KB" in v:
        v["traffic_bytes"] = round((2 * v["FETCH_SIZE_KB"] + v["WRITE_SIZE_KB"]) * 1024)
print(json.dumps({"kernel": kn, "by_grid_size": res}, indent=1))
