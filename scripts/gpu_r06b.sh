#!/bin/bash
# round 6: the sequential-id encoder's tests + the ADVICE tests, its A/B, the GPU suite, the bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_f64_enc_seq.py tests/test_gpu_api.py > gpurun_out/r06b_new.log 2>&1
rc=$?; tail -3 gpurun_out/r06b_new.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u scripts/ab_enc_f64.py r06b 10000000 100000000 > gpurun_out/r06b_ab_enc.log 2>&1
rc=$?; cat gpurun_out/r06b_ab_enc.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 $T tests > gpurun_out/r06b_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r06b_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r06b_bench.json 2> gpurun_out/r06b_bench.err
rc=$?; cut -c1-300 gpurun_out/r06b_bench.json; exit $rc
