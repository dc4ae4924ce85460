#!/bin/bash
# round 5: rocprofv3 evidence (trace + FETCH / WRITE / SQ passes) of the final mixed decode and
# archive decode at 10^7
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
scripts/profile_cmd.sh r05_mixed python3 $R/scripts/ab_mixed.py plainonly > gpurun_out/r05p_mixed.log 2>&1 || { tail -5 gpurun_out/r05p_mixed.log; exit 1; }
scripts/profile_cmd.sh r05_arch python3 $R/scripts/run_archive.py 10000000 3 > gpurun_out/r05p_arch.log 2>&1 || { tail -5 gpurun_out/r05p_arch.log; exit 1; }
echo done
