#!/bin/bash
# f64 iteration: GPU parity tests, bench with the single-pass decoder, then the two-pass one.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 20 --warmup 5} > gpurun_out/bench_1p.json 2> gpurun_out/bench_1p.err
rc=$?; cat gpurun_out/bench_1p.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_1p.err; exit $rc; }
NXG_F64_2PASS=1 timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 20 --warmup 5} > gpurun_out/bench_2p.json 2> gpurun_out/bench_2p.err
rc=$?; cat gpurun_out/bench_2p.json; exit $rc
