#!/bin/bash
# round 6 baseline: the GPU suite, then the bench line, on the round-5 code
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r06a_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r06a_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r06a_bench.json 2> gpurun_out/r06a_bench.err
rc=$?; cat gpurun_out/r06a_bench.json | cut -c1-400; exit $rc
