#!/bin/bash
# GPU parity suite, then the f64 run-decoder probe.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -5; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
bash scripts/gpu_f64r.sh
