#!/bin/bash
# round 6: the fix pass following a recount's new exit into the next tiles (NXG_FMX_FIXC) --
# mixed tests, then A/B against fixc0 on config 3 plain and with control
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_mixed_fast.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_multi.py > gpurun_out/r06y_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r06y_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do for v in base fixc0; do
  lib=$R/netidx_amd/build_ab/$v/libnxg_codec.so; [ $v = base ] && lib=$R/netidx_amd/lib/libnxg_codec.so
  NXG_LIB=$lib timeout -k 10 200 python3 -u scripts/ab_mixed.py both > gpurun_out/r06y_$v.log 2>&1 || { tail -5 gpurun_out/r06y_$v.log; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/r06y_$v.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$v', d['kind'], d['ok'], d['ms1'], d['ms2'], d['diag_after'][5])"
done; done
