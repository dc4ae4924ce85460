#!/bin/bash
# round 4: mixed decoder tests, then plain / ctl timing with the per-call diagnostics
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/mix3
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mixed_fast.py tests/test_gpu_dispatch.py tests/test_gpu_multi.py tests/test_gpu_parity.py > gpurun_out/mix3/tests.log 2>&1 || { tail -30 gpurun_out/mix3/tests.log; exit 1; }
tail -2 gpurun_out/mix3/tests.log
timeout -k 10 200 python3 scripts/ab_mixed.py diag 2>&1 | grep -v amdgpu.ids
