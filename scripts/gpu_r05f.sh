#!/bin/bash
# round 5: the encoder's GPU tests, then its A/B (look-back wave during staging; array write fast path) and stamps
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -m gpu tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_archive.py tests/test_gpu_selfhelp.py tests/test_gpu_mixed_fast.py tests/test_gpu_api.py --timeout 200 --timeout-method thread > gpurun_out/r05f_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05f_tests.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="lbw0 af3" scripts/gpu_enc2.sh || exit 1
echo "== stamps encp"
NXG_LIB=$R/netidx_amd/build_ab/encp/libnxg_codec.so timeout -k 10 120 python3 scripts/stamps_enc.py 10000000 2>&1 | grep -v amdgpu.ids || exit 1
echo "== archive count sections"
NXG_LIB=$R/netidx_amd/build_ab/fap/libnxg_codec.so timeout -k 10 150 python3 scripts/prof_fa.py 2>&1 | grep -v amdgpu.ids || exit 1
