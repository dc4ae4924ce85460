#!/bin/bash
# round 5: publisher commit with the slot bitmap: tests, then timings and its kernel split
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -m gpu tests/test_gpu_dispatch.py tests/test_gpu_publish.py --timeout 200 --timeout-method thread > gpurun_out/r05k_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r05k_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  echo "$(timeout -k 10 120 python3 scripts/diag_dispatch.py 10000000 16 seq 2>&1 | grep call=) | $(timeout -k 10 120 python3 scripts/diag_publish.py 2>&1 | grep call=)"
done
scripts/gpu_r05h.sh || exit 1
