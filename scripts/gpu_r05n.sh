#!/bin/bash
# round 5: nontemporal column stores in the mixed / archive emits: tests, then A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -m gpu tests/test_gpu_mixed_fast.py tests/test_gpu_archive.py tests/test_gpu_parity.py tests/test_gpu_multi.py --timeout 200 --timeout-method thread > gpurun_out/r05n_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r05n_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in base nt0; do
    lib=$R/netidx_amd/build_ab/$v/libnxg_codec.so
    [ $v = base ] && lib=$R/netidx_amd/lib/libnxg_codec.so
    NXG_LIB=$lib timeout -k 10 200 python3 -u scripts/ab_mixed.py $v 2>&1 | grep -v amdgpu.ids | cut -c1-170 || exit 1
  done
done
scripts/gpu_ab_arch2.sh base nt0 || exit 1
