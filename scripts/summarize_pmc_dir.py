"""Per-kernel means per dispatch from a scripts/profile_cmd.sh output directory (trace stats,
FETCH_SIZE, WRITE_SIZE, SQ counters) -> <dir>/summary.json, printed."""
import collections
import csv
import glob
import json
import sys


def kname(full):
    n = full.split("(")[0] if not full.startswith("(anonymous") else full.split("::", 1)[1].split("(")[0]
    return n.replace("void ", "")


out = sys.argv[1]
res = {}
for d in ("fetch", "write", "sq1", "sq2"):
    f = glob.glob(f"{out}/{d}/**/*counter_collection.csv", recursive=True)
    if not f:
        continue
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(f[0])):
        k = kname(r["Kernel_Name"])
        if not k.startswith("nxg"):
            continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    for k, cs in acc.items():
        n = len(disp[k])
        res.setdefault(k, {"dispatches": n}).update({c: v / n for c, v in sorted(cs.items())})
st = glob.glob(f"{out}/trace/**/*kernel_stats.csv", recursive=True)
if st:
    for r in csv.DictReader(open(st[0])):
        k = kname(r["Name"])
        if k in res or k.startswith("nxg"):
            res.setdefault(k, {})["avg_ns"] = float(r["AverageNs"])
            res[k]["calls"] = int(r["Calls"])
json.dump(res, open(f"{out}/summary.json", "w"), indent=1)
print(json.dumps(res, indent=1))
