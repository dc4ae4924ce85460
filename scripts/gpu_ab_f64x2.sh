#!/bin/bash
# A/B of single-pass f64 decoder builds (scripts/ab_variants.sh build ...): random-order ids at
# 10^7 and 10^8, kernel trace per variant, plus the decoder's GPU tests on each build
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
for name in "$@"; do
  lib=$R/netidx_amd/build_ab/$name/libnxg_codec.so
  [ "$name" = base ] && lib=$R/netidx_amd/lib/libnxg_codec.so
  cd $R
  NXG_LIB=$lib timeout -k 10 300 python -m pytest -q tests/test_gpu_fullsize.py -k "single_pass or false_record or random_order" --timeout 120 --timeout-method thread > gpurun_out/abx_${name}_tests.log 2>&1
  echo "== $name tests: $(tail -1 gpurun_out/abx_${name}_tests.log)"
  for N in 10000000 100000000; do
    OUT=$R/gpurun_out/abx_${name}_$N; rm -rf $OUT; mkdir -p $OUT
    cd /tmp
    NXG_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $R/scripts/run_f64x.py $N 10 > $OUT/run.log 2>&1 || exit 1
    f=$(find $OUT/trace -name '*kernel_stats.csv' | head -1)
    echo "$name $N $(grep -h 'n=' $OUT/run.log) $(grep f64x_kernel $f | awk -F'","' '{print $0}' | python3 -c "import sys,csv; r=list(csv.reader(sys.stdin)); print('f64x_us', round(float(r[0][3])/1000,1) if r else None)")"
  done
done
