#!/bin/bash
# round 4: sequential-id decoder A/B after the count-free XCD mapping (occupancy cap, R=8, XCD run
# lengths), the length-run decoder beside it on the same box
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/seq5
AB_PATHS=seq,run scripts/gpu_ab_f64s.sh "10000000 100000000" base 2>&1 | grep -v amdgpu.ids | tee gpurun_out/seq5/ab.log
AB_PATHS=seq scripts/gpu_ab_f64s.sh "10000000 100000000" o6 o5 o4 r8 x16 x256 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/seq5/ab.log
