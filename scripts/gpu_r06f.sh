#!/bin/bash
# round 6: partition view timing + kernel trace; mixed decode A/B (emit occupancy 5, old candidate scan)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_partition.py > gpurun_out/r06f_part.log 2>&1
rc=$?; tail -1 gpurun_out/r06f_part.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -u scripts/ab_partition.py base 2>&1 | grep -v amdgpu.ids || exit 1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r06_part -o trace -- python3 $R/scripts/ab_partition.py trace > $R/gpurun_out/r06f_part_trace.log 2>&1 || exit 1
cd $R && grep -h "part_" gpurun_out/prof_r06_part/*/trace_kernel_stats.csv 2>/dev/null | cut -c1-200
for rep in 1 2; do
  for v in base eocc5 cm1; do
    lib=$R/netidx_amd/build_ab/$v/libnxg_codec.so
    [ $v = base ] && lib=$R/netidx_amd/lib/libnxg_codec.so
    NXG_LIB=$lib timeout -k 10 200 python3 -u scripts/ab_mixed.py plainonly 2>&1 | grep -v amdgpu.ids | sed "s/plainonly/$v/" | cut -c1-200 || exit 1
  done
done
