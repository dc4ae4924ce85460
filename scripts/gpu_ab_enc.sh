#!/bin/bash
# mixed encode time (10^7 records) for library variants
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for name in "$@"; do
  lib=$R/netidx_amd/build_ab/$name/libnxg_codec.so
  [ "$name" = base ] && lib=$R/netidx_amd/lib/libnxg_codec.so
  echo "== $name"
  NXG_LIB=$lib timeout -k 10 120 python3 $R/scripts/diag_encode.py 10000000 || exit 1
done
