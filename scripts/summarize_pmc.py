"""Per-kernel means per dispatch of a scripts/prof_cmd.sh output directory -> summary.json."""
import collections
import csv
import glob
import json
import sys

out = sys.argv[1]
res = {}
for d in ("fetch", "write", "sq1", "sq2"):
    f = glob.glob(f"{out}/{d}/**/*counter_collection.csv", recursive=True)
    if not f:
        continue
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        if "nxg" not in k:
            continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    for k, cs in acc.items():
        n = len(disp[k])
        res.setdefault(k, {"dispatches": n}).update({c: v / n for c, v in sorted(cs.items())})
st = glob.glob(f"{out}/trace/**/*kernel_stats.csv", recursive=True)
if st:
    for r in csv.DictReader(open(st[0])):
        k = r["Name"].replace("(anonymous namespace)::", "").split("(")[0]
        if k in res or "nxg" in k:
            res.setdefault(k, {})["avg_ns"] = float(r["AverageNs"])
            res[k]["calls"] = int(r["Calls"])
json.dump(res, open(f"{out}/summary.json", "w"), indent=1)
for k, v in res.items():
    print(k, json.dumps({c: round(x, 1) if isinstance(x, float) else x for c, x in v.items()}))
