#!/bin/bash
# GPU suite, bench (default args), then the rocprofv3 evidence at 10^7 and 10^8.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; cat gpurun_out/bench.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench.err; exit $rc; }
bash scripts/profile_f64.sh ${TAG:-r02c} > gpurun_out/profile.log 2>&1; rc=$?; tail -5 gpurun_out/profile.log; [ $rc -eq 0 ] || exit $rc
RECORDS=100000000 bash scripts/profile_f64.sh ${TAG:-r02c}_1e8 > gpurun_out/profile_1e8.log 2>&1; rc=$?; tail -5 gpurun_out/profile_1e8.log; exit $rc
