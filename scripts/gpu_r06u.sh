#!/bin/bash
# round 6: where the dispatch count's time goes -- timing-only builds without the last_row
# atomics (sk1), the LDS counters (sk2), the row cache stores (sk4), all three (sk7)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in base sk1 sk2 sk4 sk7; do
  lib=$R/netidx_amd/build_ab/$v/libnxg_codec.so; [ $v = base ] && lib=$R/netidx_amd/lib/libnxg_codec.so
  rm -rf gpurun_out/tr_$v
  cd /tmp
  NXG_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/tr_$v -o t -- python3 $R/scripts/diag_dispatch.py 10000000 16 seq > $R/gpurun_out/tr_$v.log 2>&1 || exit 1
  cd $R
  python3 -c "
import csv,glob
f=glob.glob('gpurun_out/tr_$v/*kernel_stats.csv')[0]
print('$v', [(r['Name'].split('(')[0][:28], round(float(r['AverageNs'])/1e3,1)) for r in csv.DictReader(open(f)) if 'disp' in r['Name'] or 'fill' in r['Name']])"
done
