#!/bin/bash
# round 6: counters of the subscriber dispatch (sequential Ids, the bench's table) and the
# publisher commit, for the dispatch / publish item
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
bash scripts/profile_cmd.sh disp_seq python3 $R/scripts/diag_dispatch.py 10000000 16 seq > gpurun_out/r06p_disp.log 2>&1 || { tail -20 gpurun_out/r06p_disp.log; exit 1; }
cat gpurun_out/r06p_disp.log | tail -40
bash scripts/profile_cmd.sh pub python3 $R/scripts/diag_publish.py > gpurun_out/r06p_pub.log 2>&1 || { tail -20 gpurun_out/r06p_pub.log; exit 1; }
cat gpurun_out/r06p_pub.log | tail -60
