#!/bin/bash
# round 4 final: mixed / archive tests and timings, then the whole GPU suite, smoke() and the bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
scripts/gpu_mix3.sh || exit 1
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_archive.py > gpurun_out/ta.log 2>&1 || { tail -20 gpurun_out/ta.log; exit 1; }
tail -1 gpurun_out/ta.log
scripts/trace_arch.sh base || true
TAG=${TAG:-r04e} scripts/gpu_r04b.sh
