#!/bin/bash
# round 4 final (records per lane by frame size): seq-kernel tests and timing, then the whole GPU
# suite, smoke() and the bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/f2
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_f64_seq.py tests/test_gpu_fullsize.py > gpurun_out/f2/tests.log 2>&1 || { tail -30 gpurun_out/f2/tests.log; exit 1; }
tail -1 gpurun_out/f2/tests.log
AB_PATHS=seq timeout -k 10 300 python3 -u scripts/ab_f64s.py base 10000000 100000000 2>&1 | grep -v amdgpu.ids | cut -c1-260 || exit 1
TAG=r04f scripts/gpu_r04b.sh
