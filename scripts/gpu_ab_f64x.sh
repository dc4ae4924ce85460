#!/bin/bash
# the single-pass f64 decoder (ids in random order) for library variants, interleaved twice
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
NS=$1; shift
for rep in 1 2; do
  for name in "$@"; do
    lib=$R/netidx_amd/build_ab/$name/libnxg_codec.so
    [ "$name" = base ] && lib=$R/netidx_amd/lib/libnxg_codec.so
    AB_PERM=1 NXG_F64_PATH=x NXG_LIB=$lib timeout -k 10 240 python3 -u $R/scripts/ab_f64.py $name $NS || exit 1
  done
done
