#!/bin/bash
# rocprofv3 kernel stats of the dispatch diagnostic (each step under its own time limit)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_disp
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_disp -o run -- python3 $R/scripts/diag_dispatch.py ${N:-10000000} ${CH:-16} > $R/gpurun_out/prof_disp.log 2>&1
rc=$?; grep "n=" $R/gpurun_out/prof_disp.log; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/prof_disp.log; exit $rc; }
f=$(find $R/gpurun_out/prof_disp -name "*kernel_stats.csv" | head -1)
cut -d, -f1-4 $f | grep -i "disp\|Name\|fill\|copy"
