#!/bin/bash
# fast mixed decoder: its GPU tests, the config-3 full-size parity, then a kernel trace of the
# config-3 decode at 10^7 records
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/fmx
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_mixed_fast.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py ${EXTRA_TESTS} > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -30; exit $rc; }
timeout -k 10 120 python3 scripts/diag_general.py 1000000 10000000 > $OUT/diag.log 2>&1
rc=$?; cat $OUT/diag.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $R/scripts/diag_general.py 10000000 > $OUT/trace.log 2>&1
rc=$?
f=$(find $OUT/trace -name '*kernel_stats.csv' 2>/dev/null | head -1)
[ -n "$f" ] && grep -E "nxg_fmx|scan" "$f" | cut -d, -f1-4 | sed 's/(.*"//'
exit $rc
