#!/bin/bash
# rocprofv3 trace + counters of single-pass f64 decoder builds at 10^7 random-order ids
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for name in "$@"; do
  lib=$R/netidx_amd/build_ab/$name/libnxg_codec.so
  [ "$name" = base ] && lib=$R/netidx_amd/lib/libnxg_codec.so
  NXG_LIB=$lib scripts/profile_cmd.sh x_$name python3 $R/scripts/run_f64x.py ${N:-10000000} 10 > gpurun_out/profx_$name.log 2>&1 || { tail -20 gpurun_out/profx_$name.log; exit 1; }
  python3 - $name <<'PY'
import json,sys
d=json.load(open(f"gpurun_out/prof_x_{sys.argv[1]}/summary.json"))
for k,v in d.items():
    if "f64x" in k:
        print(sys.argv[1], k, {a: (round(b) if isinstance(b,float) else b) for a,b in v.items()})
PY
done
