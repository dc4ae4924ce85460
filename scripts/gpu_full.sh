#!/bin/bash
# smoke(), the whole GPU suite (up to 20 failures reported), then the default bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -q -m gpu --maxfail=20 --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; grep -E "^FAILED|^ERROR" gpurun_out/pytest_gpu.log | head -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc2=$?; cat gpurun_out/bench.json; [ $rc2 -eq 0 ] || { tail -5 gpurun_out/bench.err; exit $rc2; }
exit $rc
