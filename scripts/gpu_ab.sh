#!/bin/bash
# A/B of the f64 single pass against the r01e snapshot (probe), then the GPU parity suite.
set -o pipefail
mkdir -p gpurun_out
timeout -k 5 120 ./scripts/probe_f64 100000000 20 > gpurun_out/probe_1e8.log 2>&1; rc=$?
cat gpurun_out/probe_1e8.log; [ $rc -eq 0 ] || exit $rc
timeout -k 5 60 ./scripts/probe_f64 10000000 20 > gpurun_out/probe_1e7.log 2>&1; rc=$?
head -8 gpurun_out/probe_1e7.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; exit $rc
