#!/bin/bash
# round 5: A/B of the archive (fixlist, window), encoder (TLS sizing), general decoder
# (count occupancy) builds plus the dispatch split; each GPU step under its own limit
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_ab_arch2.sh base fl0 fw0 || exit 1
VARIANTS="tls0" scripts/gpu_enc2.sh || exit 1
for v in base gocc4; do
  lib=$R/netidx_amd/build_ab/$v/libnxg_codec.so
  [ $v = base ] && lib=$R/netidx_amd/lib/libnxg_codec.so
  OUT=$R/gpurun_out/abgen_$v; rm -rf $OUT; mkdir -p $OUT
  (cd /tmp && NXG_MIXED_PATH=general NXG_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats \
     --output-format csv -d $OUT/trace -o t -- python3 $R/scripts/diag_general.py 10000000 > $OUT/run.log 2>&1) || exit 1
  echo "== gen $v: $(grep -h 'n=' $OUT/run.log | cut -c1-120)"
  f=$(find $OUT/trace -name '*kernel_stats.csv' | head -1)
  cut -d, -f1-4 $f | grep -i "gen\|Name"
done
scripts/gpu_disp_prof.sh || exit 1
