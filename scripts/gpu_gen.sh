#!/bin/bash
# General-decode iteration: GPU parity tests, diag timings, rocprofv3 kernel stats of the diag.
# Every GPU step has its own time limit; steps are chained (stop at the first failure).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/diag_general.py ${DIAG_N:-100000 1000000 10000000} > gpurun_out/diag.log 2>&1
rc=$?; cat gpurun_out/diag.log; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/prof_gen
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gen -o run -- python3 scripts/diag_general.py 10000000 > gpurun_out/prof_gen.log 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/prof_gen.log; exit $rc; }
find gpurun_out/prof_gen -name "*kernel_stats.csv" | head -1 | xargs cut -d, -f1-4 | head -12
