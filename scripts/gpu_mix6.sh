#!/bin/bash
# round 4: the fix pass with several tiles per wave: mixed tests, then A/B of tiles per wave
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/mix6
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mixed_fast.py tests/test_gpu_dispatch.py tests/test_gpu_multi.py tests/test_gpu_parity.py > gpurun_out/mix6/tests.log 2>&1 || { tail -30 gpurun_out/mix6/tests.log; exit 1; }
tail -1 gpurun_out/mix6/tests.log
for rep in 1 2; do
  for v in base fixt1 fixt16; do
    lib=$R/netidx_amd/build_ab/$v/libnxg_codec.so
    [ $v = base ] && lib=$R/netidx_amd/lib/libnxg_codec.so
    NXG_LIB=$lib timeout -k 10 200 python3 -u scripts/ab_mixed.py $v 2>&1 | grep -v amdgpu.ids | cut -c1-140 || exit 1
  done
done
