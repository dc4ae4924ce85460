#!/bin/bash
# round 5: the final validation (GPU suite, smoke, bench, N=2 rehearsal)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05w} scripts/gpu_r05_final2.sh || exit 1
