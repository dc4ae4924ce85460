#!/bin/bash
# A/B of fast mixed decoder builds (scripts/ab_variants.sh build ...): config-3 decode at 10^7,
# kernel trace per variant; diag_general prints DevStatus.diag (4: waves that waited on the
# previous wave's exit, 5: tiles recounted by the resolve pass)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
for name in "$@"; do
  lib=$R/netidx_amd/build_ab/$name/libnxg_codec.so
  [ "$name" = base ] && lib=$R/netidx_amd/lib/libnxg_codec.so
  OUT=$R/gpurun_out/abfmx_$name; rm -rf $OUT; mkdir -p $OUT
  cd /tmp
  NXG_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $R/scripts/diag_general.py 10000000 > $OUT/diag.log 2>&1 || exit 1
  f=$(find $OUT/trace -name '*kernel_stats.csv' | head -1)
  echo "== $name"; grep -v amdgpu.ids $OUT/diag.log | cut -c1-300
  grep fmx "$f" | cut -d, -f1,2,4 | sed 's/(.*)"//'
done
