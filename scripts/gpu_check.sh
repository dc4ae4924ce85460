#!/bin/bash
# One GPU-box pass: parity tests, smoke, a short bench. Every GPU step has its own time limit
# and the steps are chained with && (stop at the first failure).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 \
  && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
  && timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 20 --warmup 5} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
tail -5 gpurun_out/pytest_gpu.log
exit $rc
