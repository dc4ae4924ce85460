#!/bin/bash
# one kernel trace (with stats) of the whole bench, extras included: every kernel's mean duration
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03}
OUT=$R/gpurun_out/trace_all_$TAG
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $R/bench.py --steps 40 --cpu-seconds 0.5 > $OUT/bench.json 2> $OUT/bench.err
rc=$?
f=$(find $OUT/trace -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && cp "$f" $OUT/kernel_stats.csv && cut -d, -f1-4 "$f" | cut -c1-160 | head -60
exit $rc
