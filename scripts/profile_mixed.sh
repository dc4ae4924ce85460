#!/bin/bash
# rocprofv3 evidence for the mixed (general) decode at config 3 (10^7 records), run on the GPU box
# from the repo root: a kernel trace with stats, then FETCH_SIZE, WRITE_SIZE and two SQ counter
# groups, each pass its own run under its own time limit. Writes gpurun_out/prof_mixed_$TAG/ and
# the per-kernel means per dispatch to gpurun_out/prof_mixed_$TAG/summary.json.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02}
N=${RECORDS:-10000000}
export TMPDIR=/tmp
OUT=$R/gpurun_out/prof_mixed_$TAG
rm -rf $OUT
mkdir -p $OUT
cd /tmp
P="python3 $R/scripts/diag_general.py $N"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- $P > $OUT/trace.log 2>&1 \
 && timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $P > $OUT/fetch.log 2>&1 \
 && timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $P > $OUT/write.log 2>&1 \
 && timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES --output-format csv -d $OUT/sq1 -o run -- $P > $OUT/sq1.log 2>&1 \
 && timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH --output-format csv -d $OUT/sq2 -o run -- $P > $OUT/sq2.log 2>&1 \
 && cd $R && python3 - "$OUT" <<'PY'
import csv, glob, collections, json, sys
out = sys.argv[1]
res = {}
for d in ("fetch", "write", "sq1", "sq2"):
    f = glob.glob(f"{out}/{d}/**/*counter_collection.csv", recursive=True)
    if not f:
        continue
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"].split("(")[0]
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
        k = r["Name"].split("(")[0]
        if k in res or k.startswith("nxg"):
            res.setdefault(k, {})["avg_ns"] = float(r["AverageNs"])
            res[k]["calls"] = int(r["Calls"])
json.dump(res, open(f"{out}/summary.json", "w"), indent=1)
print(json.dumps(res, indent=1))
PY
