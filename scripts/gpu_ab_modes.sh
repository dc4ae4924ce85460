#!/bin/bash
# stream-of-frames vs one call per frame at 10^8 (and 10^7), per library build, interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for rep in 1 2; do
  for name in "$@"; do
    lib=$R/netidx_amd/build_ab/$name/libnxg_codec.so
    [ "$name" = base ] && lib=$R/netidx_amd/lib/libnxg_codec.so
    for N in 100000000 10000000; do
      NXG_LIB=$lib timeout -k 10 200 python3 $R/scripts/run_f64_modes.py $N 20 2>/dev/null | tail -2 | sed "s/^/$name rep$rep /" || exit 1
    done
  done
done
