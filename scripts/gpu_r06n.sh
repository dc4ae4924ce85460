#!/bin/bash
# round 6: where the mixed emit's VALU goes -- SQ_INSTS_VALU / time of timing-only builds that skip
# one section each (NXG_FMX_SKIP: 1 elements, 2 text checks, 4 row values, 8 row stores)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in base skip1 skip2 skip4 skip8; do
  lib=$R/netidx_amd/build_ab/$v/libnxg_codec.so; [ $v = base ] && lib=$R/netidx_amd/lib/libnxg_codec.so
  OUT=$R/gpurun_out/pmc_emit_$v; rm -rf $OUT; mkdir -p $OUT
  cd /tmp
  NXG_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES --output-format csv -d $OUT -o run -- python3 $R/scripts/ab_mixed.py plainonly > $OUT/log 2>&1 || exit 1
  cd $R
  python3 - $OUT $v <<'PY'
import csv, glob, collections, sys
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); disp = collections.defaultdict(set)
for r in csv.DictReader(open(f)):
    if "fmx_emit" in r["Kernel_Name"]:
        acc["e"][r["Counter_Name"]] += float(r["Counter_Value"]); disp["e"].add(r["Dispatch_Id"])
n = len(disp["e"]); c = acc["e"]
print(sys.argv[2], {k: round(v / n / 1e6, 2) for k, v in c.items()})
PY
done
