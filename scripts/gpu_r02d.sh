#!/bin/bash
# GPU suite, bench (default args), then a kernel trace of the config-3 mixed decode at 10^7.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; cat gpurun_out/bench.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench.err; exit $rc; }
mkdir -p gpurun_out/mx
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/mx/trace -o trace -- python3 $R/scripts/diag_general.py 10000000 > $R/gpurun_out/mx/trace.log 2>&1
rc=$?
f=$(find $R/gpurun_out/mx/trace -name '*kernel_stats.csv' 2>/dev/null | head -1)
[ -n "$f" ] && cut -d, -f1-6 "$f" | head -30
exit $rc
