#!/bin/bash
# f64 decoder A/B on the GPU box: scripts/gpu_ab_f64s.sh "N1 N2" base name2 ...
# (base: netidx_amd/lib; others: netidx_amd/build_ab/<name>), two interleaved rounds.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
NS=$1; shift
mkdir -p $R/gpurun_out
for rep in 1 2; do
  for name in "$@"; do
    lib=$R/netidx_amd/build_ab/$name/libnxg_codec.so
    [ "$name" = base ] && lib=$R/netidx_amd/lib/libnxg_codec.so
    NXG_LIB=$lib timeout -k 10 240 python3 -u $R/scripts/ab_f64s.py $name $NS || exit 1
  done
done
