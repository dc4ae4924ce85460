#!/bin/bash
# round 6: the GPU suite, the partition view (unrolled ranking) timing + trace, the bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread"
timeout -k 10 700 $T tests > gpurun_out/r06k_pytest.log 2>&1
rc=$?; tail -1 gpurun_out/r06k_pytest.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r06_part3 -o trace -- python3 $R/scripts/ab_partition.py trace > $R/gpurun_out/r06k_part_trace.log 2>&1 || exit 1
cd $R && grep -v amdgpu.ids gpurun_out/r06k_part_trace.log | grep '"tag"'
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof_r06_part3/trace_kernel_stats.csv')):
    if 'part_' in r['Name']: print(r['Name'].split('(')[0], r['Calls'], r['AverageNs'], r['MinNs'])"
timeout -k 10 700 python -u bench.py > gpurun_out/r06k_bench.json 2> gpurun_out/r06k_bench.err
rc=$?; cut -c1-200 gpurun_out/r06k_bench.json; exit $rc
