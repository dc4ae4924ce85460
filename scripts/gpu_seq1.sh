#!/bin/bash
# round 4: first look at the sequential-id decoder: its tests, then the A/B against the length-run
# decoder and the build variants (R=2, nontemporal stores / loads)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/seq1
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_f64_seq.py > gpurun_out/seq1/tests.log 2>&1 || { tail -30 gpurun_out/seq1/tests.log; exit 1; }
tail -3 gpurun_out/seq1/tests.log
scripts/gpu_ab_f64s.sh "10000000 100000000" base r2 nt1 nt2 2>&1 | grep -v amdgpu.ids | tee gpurun_out/seq1/ab.log
