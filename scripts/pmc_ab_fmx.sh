#!/bin/bash
# SQ instruction counters of the fast mixed emit kernel (config 3, 10^7) for library variants
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
for name in "$@"; do
  lib=$R/netidx_amd/build_ab/$name/libnxg_codec.so
  [ "$name" = base ] && lib=$R/netidx_amd/lib/libnxg_codec.so
  OUT=$R/gpurun_out/pmcab/$name
  rm -rf $OUT; mkdir -p $OUT
  (cd /tmp && NXG_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT -o run -- python3 $R/scripts/diag_general.py 10000000 > $OUT/log 2>&1) || { tail -5 $OUT/log; exit 1; }
  python3 - $OUT $name <<'PY'
import csv, glob, collections, os, sys
KN = os.environ.get("KN", "nxg_fmx_emit")
acc = collections.defaultdict(float)
for f in glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith(KN):
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
w = acc.pop("SQ_WAVES", 1)
print(sys.argv[2], " ".join(f"{k[3:]}={v / w:.0f}" for k, v in sorted(acc.items())))
PY
done
