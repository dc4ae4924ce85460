#!/bin/bash
# Build variants of the library into netidx_amd/build_ab/<name>/ (here, CPU side):
#   scripts/ab_variants.sh build name "-DFLAG=.." [name2 "-D.."] ...
# and time them on the GPU box (bench at 10^7 and 10^8, interleaved, kernel-event times):
#   scripts/ab_variants.sh run name name2 ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cmd=$1; shift
if [ "$cmd" = build ]; then
  while [ $# -ge 2 ]; do
    name=$1; flags=$2; shift 2
    make -C $R/netidx_amd/csrc -s OBJDIR=../build_ab/$name/obj OUTDIR=../build_ab/$name \
      CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-variable -munsafe-fp-atomics $flags" || exit 1
  done
  exit 0
fi
for rep in ${REPS:-1 2}; do
  for name in "$@"; do
    for N in 10000000 100000000; do
      lib=$R/netidx_amd/build_ab/$name/libnxg_codec.so
      [ "$name" = base ] && lib=$R/netidx_amd/lib/libnxg_codec.so
      NXG_LIB=$lib timeout -k 10 200 python3 $R/bench.py --steps 40 --warmup 3 --no-extras --cpu-seconds 0.1 --records $N > $R/gpurun_out/ab_${name}_${N}_$rep.json 2>/dev/null || exit 1
      python3 -c "
import json,sys
d=json.loads(open('$R/gpurun_out/ab_${name}_${N}_$rep.json').read().strip().splitlines()[-1])
print('$name', $N, 'rep $rep', 'kernel_ms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'], flush=True)"
    done
  done
done
