#!/bin/bash
# kernel trace of the archive batch decode (10^7 items) for library variants
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
for name in "$@"; do
  lib=$R/netidx_amd/build_ab/$name/libnxg_codec.so
  [ "$name" = base ] && lib=$R/netidx_amd/lib/libnxg_codec.so
  OUT=$R/gpurun_out/trarch/$name; rm -rf $OUT; mkdir -p $OUT
  (cd /tmp && NXG_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o t -- python3 $R/scripts/diag_archive.py 10000000 > $OUT/log 2>&1) || { tail -3 $OUT/log; exit 1; }
  echo "== $name"; python3 $R/scripts/kstats.py $(find $OUT -name '*kernel_stats.csv' | head -1) | grep arch
done
