#!/bin/bash
# round 4: general encoder variants (scripts/ab_variants.sh build ...), config 3 at 10^7
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/enc2
for rep in 1 2; do
  for v in base ${VARIANTS:-eb1 eb8 nolb}; do
    lib=$R/netidx_amd/build_ab/$v/libnxg_codec.so
    [ $v = base ] && lib=$R/netidx_amd/lib/libnxg_codec.so
    echo -n "$v: "
    NXG_LIB=$lib timeout -k 10 200 python3 -u scripts/diag_encode.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/enc2/ab.log || exit 1
  done
done
