#!/bin/bash
# two SQ counter passes over the config-3 decode (10^7 records), nxg kernels summarised per wave
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_fmx_${1:-x}
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
P="python3 $R/scripts/diag_general.py 10000000"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/a -o run -- $P > $OUT/a.log 2>&1 \
 && timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES --output-format csv -d $OUT/b -o run -- $P > $OUT/b.log 2>&1
rc=$?
cd $R && python3 - "$OUT" <<'PY'
import csv, glob, collections, sys
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for d in ("a", "b"):
    for f in glob.glob(f"{out}/{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            if k.startswith("nxg_fmx"):
                acc[k][r["Counter_Name"] + "@" + d] += float(r["Counter_Value"])
for k, cs in acc.items():
    waves = cs.get("SQ_WAVES@a", 1)
    print(k, "waves", waves)
    for c, v in sorted(cs.items()):
        if not c.startswith("SQ_WAVES"):
            print(f"   {c:28s} {v:14.0f}  per wave {v / waves:10.1f}")
PY
exit $rc
