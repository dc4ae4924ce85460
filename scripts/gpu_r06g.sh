#!/bin/bash
# round 6: partition view (values loaded up front) + trace; mixed decode A/B: class-branched emit
# at 5 waves/SIMD (8 B/lane spill) vs val_decode at 5 waves/SIMD (no spill)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_partition.py tests/test_gpu_mixed_fast.py > gpurun_out/r06g_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r06g_tests.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r06_part2 -o trace -- python3 $R/scripts/ab_partition.py trace > $R/gpurun_out/r06g_part_trace.log 2>&1 || exit 1
cd $R && grep -v amdgpu.ids gpurun_out/r06g_part_trace.log | grep '"tag"'
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof_r06_part2/trace_kernel_stats.csv')):
    if 'part_' in r['Name']: print(r['Name'].split('(')[0], r['Calls'], r['AverageNs'], r['MinNs'])"
for rep in 1 2 3; do
  for v in base c0e5; do
    lib=$R/netidx_amd/build_ab/$v/libnxg_codec.so
    [ $v = base ] && lib=$R/netidx_amd/lib/libnxg_codec.so
    NXG_LIB=$lib timeout -k 10 200 python3 -u scripts/ab_mixed.py plainonly 2>&1 | grep -v amdgpu.ids | sed "s/plainonly/$v/" | cut -c1-160 || exit 1
  done
done
