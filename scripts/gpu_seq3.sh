#!/bin/bash
# round 4: sequential-id decoder A/B (occupancy caps, R=8, no XCD remap), all with NT stores
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/${AB_OUT:-seq3}
AB_PATHS=seq scripts/gpu_ab_f64s.sh "10000000 100000000" ${AB_VARIANTS:-nt1} 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${AB_OUT:-seq3}/ab.log
