#!/bin/bash
# kernel trace + stats only: scripts/gpu_trace.sh TAG cmd...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
export TMPDIR=/tmp
OUT=$R/gpurun_out/trace_$TAG
rm -rf $OUT; mkdir -p $OUT
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o trace -- "$@" > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
cd $R
python3 - $OUT <<'PY'
import csv,sys,glob
f=glob.glob(sys.argv[1]+"/**/trace_kernel_stats.csv",recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(r["Name"][:60], "calls", r["Calls"], "avg_us", round(float(r["AverageNs"])/1000,1), "min_us", round(float(r["MinNs"])/1000,1), "max_us", round(float(r["MaxNs"])/1000,1))
PY
