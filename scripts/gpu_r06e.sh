#!/bin/bash
# round 6: the type-partitioned view's tests, then rocprofv3 evidence (mixed decoder: this
# round's build and the round-5 variant; the sequential-id f64 encoder's writing launches; the
# random-order f64 decoder), then the bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_partition.py > gpurun_out/r06e_part.log 2>&1
rc=$?; tail -3 gpurun_out/r06e_part.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r06d.sh || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/r06e_bench.json 2> gpurun_out/r06e_bench.err
rc=$?; cut -c1-300 gpurun_out/r06e_bench.json; exit $rc
