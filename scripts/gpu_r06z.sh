#!/bin/bash
# round 6: partition tiles of 4096 (base) / 2048 / 1024 rows -- partition tests per build, A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread"
for v in t2k t1k; do
  NXG_LIB=$R/netidx_amd/build_ab/$v/libnxg_codec.so timeout -k 10 300 $T tests/test_gpu_partition.py > gpurun_out/r06z_$v.log 2>&1; rc=$?; echo -n "$v tests: "; tail -1 gpurun_out/r06z_$v.log; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2 3; do for v in base t2k t1k; do
  lib=$R/netidx_amd/build_ab/$v/libnxg_codec.so; [ $v = base ] && lib=$R/netidx_amd/lib/libnxg_codec.so
  echo -n "$v rep$rep: "; NXG_LIB=$lib timeout -k 10 200 python3 -u scripts/ab_partition.py $v 2>&1 | grep -v amdgpu.ids | tail -1 | cut -c1-200 || exit 1
done; done
