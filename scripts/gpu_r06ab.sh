#!/bin/bash
# round 6: dispatch segments of 256 rows, one per wave (base) against the round-5 1024-row
# segments on a capped grid (v1024) and two neighbours; dispatch + publish tests first
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread"
NXG_LIB=$R/netidx_amd/build_ab/g16/libnxg_codec.so timeout -k 10 400 $T tests/test_gpu_publish.py > gpurun_out/r06q_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r06q_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do for v in base g4 g16; do
  lib=$R/netidx_amd/build_ab/$v/libnxg_codec.so; [ $v = base ] && lib=$R/netidx_amd/lib/libnxg_codec.so
  for o in seq random; do
    echo -n "$v rep$rep: "; NXG_LIB=$lib timeout -k 10 120 python3 -u scripts/diag_dispatch.py 10000000 16 $o 2>&1 | grep "n=" || exit 1
  done
  echo -n "$v rep$rep pub: "; NXG_LIB=$lib timeout -k 10 120 python3 -u scripts/diag_publish.py 2>&1 | grep "n=" || exit 1
done; done
