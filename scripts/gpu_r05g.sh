#!/bin/bash
# round 5: archive count (chain loop skips synchronised chunks, run tails with arrays): tests,
# A/B and section clocks; each GPU step under its own limit
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -m gpu tests/test_gpu_archive.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py --timeout 200 --timeout-method thread > gpurun_out/r05g_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05g_tests.log; [ $rc -eq 0 ] || exit $rc
scripts/gpu_ab_arch2.sh base fa10 fa00 || exit 1
echo "== archive count sections"
NXG_LIB=$R/netidx_amd/build_ab/fap/libnxg_codec.so timeout -k 10 150 python3 scripts/prof_fa.py 2>&1 | grep -v amdgpu.ids || exit 1
