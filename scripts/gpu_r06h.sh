#!/bin/bash
# round 6: archive emit at 5 waves/SIMD (A/B, kernel traces), then the bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread"
NXG_LIB=$R/netidx_amd/build_ab/fae5/libnxg_codec.so timeout -k 10 400 $T tests/test_gpu_archive.py > gpurun_out/r06h_arch_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r06h_arch_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab_arch2.sh base fae5 base fae5 || exit 1
for rep in 1 2; do for v in base keep; do
  lib=$R/netidx_amd/build_ab/$v/libnxg_codec.so; [ $v = base ] && lib=$R/netidx_amd/lib/libnxg_codec.so
  NXG_LIB=$lib timeout -k 10 200 python3 -u scripts/ab_enc_mixed.py $v 2>&1 | grep -v amdgpu.ids || exit 1
done; done
cd $R && timeout -k 10 600 python -u bench.py > gpurun_out/r06h_bench.json 2> gpurun_out/r06h_bench.err
rc=$?; cut -c1-200 gpurun_out/r06h_bench.json; exit $rc
