#!/bin/bash
# A/B of single-pass f64 decoder builds (scripts/ab_variants.sh build ...): the decoder's GPU tests
# on each build, then random-order timing at 10^7 (3 frames in rotation) and 10^8 (2 frames),
# HIP events on the codec stream (scripts/ab_f64x.py), interleaved over REPS rounds
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
lib_of() { [ "$1" = base ] && echo $R/netidx_amd/lib/libnxg_codec.so || echo $R/netidx_amd/build_ab/$1/libnxg_codec.so; }
for name in "$@"; do
  NXG_LIB=$(lib_of $name) timeout -k 10 300 python -m pytest -q tests/test_gpu_fullsize.py tests/test_gpu_selfhelp.py tests/test_gpu_multi.py -k "single_pass or false_record or random_order or selfhelp or patience or two_processes" --timeout 120 --timeout-method thread > gpurun_out/abx3_${name}_tests.log 2>&1
  rc=$?
  echo "== $name tests: $(tail -1 gpurun_out/abx3_${name}_tests.log)"
  [ $rc -ne 0 ] && exit 1
done
for rep in ${REPS:-1 2}; do
  for name in "$@"; do
    NXG_LIB=$(lib_of $name) timeout -k 10 200 python3 scripts/ab_f64x.py $name ${SIZES:-10000000 100000000} 2>/dev/null || exit 1
  done
done
