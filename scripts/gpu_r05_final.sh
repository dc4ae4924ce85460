#!/bin/bash
# round 5 final: the whole GPU suite, smoke(), the default bench line, then rocprofv3 evidence of
# the bench command (headline legs only: kernel trace + FETCH / WRITE / SQ passes)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
TAG=${TAG:-r05z} scripts/gpu_r04b.sh || exit 1
scripts/profile_cmd.sh ${TAG:-r05z}_bench python3 $R/bench.py --no-extras --cpu-seconds 2 --steps 100 || exit 1
tail -3 gpurun_out/prof_${TAG:-r05z}_bench/trace.log
scripts/gpu_r05h.sh || exit 1
