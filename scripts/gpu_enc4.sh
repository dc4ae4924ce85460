#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 200 python3 -u scripts/diag_enc_diff.py 50000 55 2>&1 | grep -v amdgpu.ids || exit 1
mkdir -p gpurun_out/enc3
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_archive.py tests/test_gpu_selfhelp.py tests/test_gpu_api.py -k "enc or arch or selfhelp or round" > gpurun_out/enc3/tests.log 2>&1 || { tail -30 gpurun_out/enc3/tests.log; exit 1; }
tail -2 gpurun_out/enc3/tests.log
for rep in 1 2; do
  timeout -k 10 200 python3 -u scripts/diag_encode.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/enc3/time.log || exit 1
done
