#!/bin/bash
# round 5: the GPU suite on the current library, then the encoder A/B (next-entry prefetch) and
# its phase stamps; each GPU step under its own limit
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -m gpu tests --timeout 300 --timeout-method thread > gpurun_out/r05e_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05e_tests.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="pf0" scripts/gpu_enc2.sh || exit 1
echo "== stamps encp"
NXG_LIB=$R/netidx_amd/build_ab/encp/libnxg_codec.so timeout -k 10 120 python3 scripts/stamps_enc.py 10000000 2>&1 | grep -v amdgpu.ids || exit 1
