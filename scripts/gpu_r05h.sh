#!/bin/bash
# round 5: kernel splits of the subscriber dispatch (sequential ids, as the bench) and the
# publisher commit; each GPU step under its own limit
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
for job in "disp python3 $R/scripts/diag_dispatch.py 10000000 16 seq" "pub python3 $R/scripts/diag_publish.py"; do
  set -- $job; tag=$1; shift
  OUT=$R/gpurun_out/r05h_$tag; rm -rf $OUT; mkdir -p $OUT
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o t -- "$@" > $OUT/run.log 2>&1) || { tail -5 $OUT/run.log; exit 1; }
  echo "== $tag: $(grep -v amdgpu $OUT/run.log | grep -i "ms\|n=" | tail -2)"
  python3 - $(find $OUT/trace -name '*kernel_stats.csv' | head -1) <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print('  ', r['Name'].split('(')[0][:50], r['Calls'], round(float(r['AverageNs']) / 1000, 1))
PY
done
