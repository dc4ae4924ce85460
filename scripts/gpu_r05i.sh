#!/bin/bash
# round 5: archive fix pass following cascades (one pass vs two): tests on each build, A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in c4p1; do
  NXG_LIB=$R/netidx_amd/build_ab/$v/libnxg_codec.so timeout -k 10 300 python -u -m pytest -x -q -m gpu tests/test_gpu_archive.py --timeout 200 --timeout-method thread > gpurun_out/r05i_$v.log 2>&1
  rc=$?; echo "$v: $(tail -1 gpurun_out/r05i_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
scripts/gpu_ab_arch2.sh base c4p1 c4p2 || exit 1
