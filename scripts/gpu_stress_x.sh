#!/bin/bash
# stress of single-pass f64 decoder builds at 10^8 (K decodes each, every one checked), with the
# default look-back patience and with self-help disabled (patience 10^9)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
lib_of() { [ "$1" = base ] && echo $R/netidx_amd/lib/libnxg_codec.so || echo $R/netidx_amd/build_ab/$1/libnxg_codec.so; }
for name in "$@"; do
  echo "== $name default patience"
  NXG_LIB=$(lib_of $name) timeout -k 10 200 python3 scripts/stress_f64x.py ${N:-100000000} ${K:-40} 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== $name no self-help"
  NXG_LOOKBACK_PATIENCE=1000000000 NXG_LIB=$(lib_of $name) timeout -k 10 200 python3 scripts/stress_f64x.py ${N:-100000000} ${K:-40} 2>&1 | grep -v amdgpu.ids || exit 1
done
