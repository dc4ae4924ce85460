#!/bin/bash
# round 5: nontemporal dispatch entries: tests, then A/B (dispatch and publish)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -m gpu tests/test_gpu_dispatch.py tests/test_gpu_publish.py --timeout 200 --timeout-method thread > gpurun_out/r05o_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r05o_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for v in base dnt0; do
    lib=$R/netidx_amd/build_ab/$v/libnxg_codec.so
    [ $v = base ] && lib=$R/netidx_amd/lib/libnxg_codec.so
    echo "$v: $(NXG_LIB=$lib timeout -k 10 120 python3 scripts/diag_dispatch.py 10000000 16 seq 2>&1 | grep call=) | $(NXG_LIB=$lib timeout -k 10 120 python3 scripts/diag_publish.py 2>&1 | grep call=)"
  done
done
