#!/bin/bash
# round 6: the lean count's message walk from one window (A/B), with the mixed tests first
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_mixed_fast.py tests/test_gpu_fullsize.py -k "mixed or config3" tests/test_gpu_multi.py tests/test_gpu_parity.py > gpurun_out/r06m_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r06m_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do for v in base lm0; do
  lib=$R/netidx_amd/build_ab/$v/libnxg_codec.so; [ $v = base ] && lib=$R/netidx_amd/lib/libnxg_codec.so
  NXG_LIB=$lib timeout -k 10 200 python3 -u scripts/ab_mixed.py plainonly 2>&1 | grep -v amdgpu.ids | sed "s/plainonly/$v/" | cut -c1-175 || exit 1
done; done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r06m -o trace -- python3 $R/scripts/ab_mixed.py plainonly > /dev/null 2>&1 || exit 1
cd $R && python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof_r06m/trace_kernel_stats.csv')):
    if 'fmx' in r['Name']: print(r['Name'].split('(')[0], r['Calls'], r['AverageNs'])"
