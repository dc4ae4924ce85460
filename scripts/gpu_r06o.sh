#!/bin/bash
# round 6: the mixed emit's Array elements gathered over rounds (NXG_FMX_DEFER) -- mixed tests,
# then A/B: d0 (per round), dinl (walk inlined), base (walk out of line)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_mixed_fast.py tests/test_gpu_fullsize.py -k "mixed or config3 or deferred or array" tests/test_gpu_parity.py > gpurun_out/r06o_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r06o_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do for v in base d0 dinl; do
  lib=$R/netidx_amd/build_ab/$v/libnxg_codec.so; [ $v = base ] && lib=$R/netidx_amd/lib/libnxg_codec.so
  NXG_LIB=$lib timeout -k 10 200 python3 -u scripts/ab_mixed.py both 2>&1 | grep -v amdgpu.ids | sed "s/both/$v/" | cut -c1-175 || exit 1
done; done
