#!/bin/bash
# round 6: the mixed decoder's fix pass with a lane per tile (A/B, plain and control frames)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_mixed_fast.py tests/test_gpu_fullsize.py -k "mixed or config3" tests/test_gpu_multi.py > gpurun_out/r06l_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r06l_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do for v in base fixw0; do
  lib=$R/netidx_amd/build_ab/$v/libnxg_codec.so; [ $v = base ] && lib=$R/netidx_amd/lib/libnxg_codec.so
  NXG_LIB=$lib timeout -k 10 200 python3 -u scripts/ab_mixed.py $v 2>&1 | grep -v amdgpu.ids | cut -c1-175 || exit 1
done; done
NXG_LIB=$R/netidx_amd/lib/libnxg_codec.so timeout -k 10 400 $T tests/test_gpu_archive.py > gpurun_out/r06l_arch_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r06l_arch_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab_arch2.sh base fixw0 base fixw0 || exit 1
