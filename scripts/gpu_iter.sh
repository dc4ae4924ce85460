#!/bin/bash
# Iteration run: GPU parity tests, general-path diagnostics, bench. Chained with && (stop at
# the first failure); every step bounded by its own timeout.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/diag_general.py ${DIAG_N:-100000 1000000 10000000} > gpurun_out/diag.log 2>&1
rc=$?; cat gpurun_out/diag.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 20 --warmup 5} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err; exit $rc
