#!/bin/bash
# round 4: single-pass f64 decoder variants (scripts/ab_variants.sh build ...), random-order ids
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/f64x_ab
for rep in 1 2; do
  for v in base ${VARIANTS}; do
    lib=$R/netidx_amd/build_ab/$v/libnxg_codec.so
    [ $v = base ] && lib=$R/netidx_amd/lib/libnxg_codec.so
    NXG_LIB=$lib timeout -k 10 300 python3 -u scripts/ab_f64x.py $v ${SIZES} 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/f64x_ab/ab.log || exit 1
  done
done
