#!/bin/bash
# round 6: the GPU suite, mixed decode A/B (class-branched emit, b128 candidate scan), the bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread"
timeout -k 10 700 $T tests > gpurun_out/r06c_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r06c_pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in base cls0 cm1 old; do
    lib=$R/netidx_amd/build_ab/$v/libnxg_codec.so
    [ $v = base ] && lib=$R/netidx_amd/lib/libnxg_codec.so
    NXG_LIB=$lib timeout -k 10 200 python3 -u scripts/ab_mixed.py $v 2>&1 | grep -v amdgpu.ids | cut -c1-200 || exit 1
  done
done
timeout -k 10 600 python -u bench.py > gpurun_out/r06c_bench.json 2> gpurun_out/r06c_bench.err
rc=$?; cut -c1-300 gpurun_out/r06c_bench.json; exit $rc
