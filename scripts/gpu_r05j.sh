#!/bin/bash
# round 5: dispatch with 1 / 2 / 4 steps' lookups in flight (tests, then timings of the dispatch
# and the publisher commit), and the archive fix pass following cascades
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -m gpu tests/test_gpu_dispatch.py tests/test_gpu_publish.py --timeout 200 --timeout-method thread > gpurun_out/r05j_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r05j_tests.log; [ $rc -eq 0 ] || exit $rc
for v in du4; do
  NXG_LIB=$R/netidx_amd/build_ab/$v/libnxg_codec.so timeout -k 10 300 python -u -m pytest -x -q -m gpu tests/test_gpu_dispatch.py tests/test_gpu_publish.py --timeout 200 --timeout-method thread > gpurun_out/r05j_$v.log 2>&1
  rc=$?; echo "$v: $(tail -1 gpurun_out/r05j_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do
  for v in base du1 du4; do
    lib=$R/netidx_amd/build_ab/$v/libnxg_codec.so
    [ $v = base ] && lib=$R/netidx_amd/lib/libnxg_codec.so
    echo "$v: $(NXG_LIB=$lib timeout -k 10 120 python3 scripts/diag_dispatch.py 10000000 16 seq 2>&1 | grep call=) | $(NXG_LIB=$lib timeout -k 10 120 python3 scripts/diag_publish.py 2>&1 | grep call=)"
  done
done
scripts/gpu_r05i.sh || exit 1
