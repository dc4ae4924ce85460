#!/bin/bash
# round 6: kernel traces of the dispatch (sequential Ids) and of config 3 with control messages
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/tr_disp gpurun_out/tr_ctl
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/tr_disp -o t -- python3 $R/scripts/diag_dispatch.py 10000000 16 seq > $R/gpurun_out/tr_disp.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/tr_ctl -o t -- python3 $R/scripts/ab_mixed.py ctlonly > $R/gpurun_out/tr_ctl.log 2>&1 || exit 1
cd $R
for d in tr_disp tr_ctl; do
  f=$(find gpurun_out/$d -name "*kernel_stats.csv" | head -1)
  echo "== $d"; cut -d, -f1-4 $f | head -14
done
