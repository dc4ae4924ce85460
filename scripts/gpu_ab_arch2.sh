#!/bin/bash
# A/B of archive fast-path builds: kernel trace of 10^7 items per variant (run_archive.py)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
for name in "$@"; do
  lib=$R/netidx_amd/build_ab/$name/libnxg_codec.so
  [ "$name" = base ] && lib=$R/netidx_amd/lib/libnxg_codec.so
  OUT=$R/gpurun_out/abarch_$name; rm -rf $OUT; mkdir -p $OUT
  cd /tmp
  NXG_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o t -- python3 $R/scripts/run_archive.py 10000000 5 > $OUT/run.log 2>&1 || exit 1
  f=$(find $OUT/trace -name '*kernel_stats.csv' | head -1)
  echo "== $name $(grep -h 'n=' $OUT/run.log)"
  python3 - $f <<'PY'
import csv, sys
tot = 0
for r in csv.DictReader(open(sys.argv[1])):
    if 'fa_' in r['Name']:
        us = float(r['AverageNs']) / 1000 * int(r['Calls']) / 5
        tot += us
        print(' ', r['Name'].split('(')[0], round(us, 1))
print('  total per decode', round(tot, 1))
PY
done
