#!/bin/bash
# kernel times of the fast mixed decoder (config 3, 10^7 records) for library variants:
#   scripts/gpu_ab_fmx.sh base old skip1 ...   (base: netidx_amd/lib; others: netidx_amd/build_ab/<name>)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
for name in "$@"; do
  lib=$R/netidx_amd/build_ab/$name/libnxg_codec.so
  [ "$name" = base ] && lib=$R/netidx_amd/lib/libnxg_codec.so
  OUT=$R/gpurun_out/abfmx/$name
  rm -rf $OUT; mkdir -p $OUT
  (cd /tmp && NXG_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o t -- python3 $R/scripts/diag_general.py 10000000 > $OUT/log 2>&1) || { tail -5 $OUT/log; exit 1; }
  f=$(find $OUT -name '*kernel_stats.csv' | head -1)
  echo "== $name"; python3 $R/scripts/kstats.py $f | grep fmx
done
