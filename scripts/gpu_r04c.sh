#!/bin/bash
# round 4: f64 decoder traces + counters at 10^8 / 10^7 (sequential-id kernel and length-run path),
# and the single-pass decoder on random-order ids at 10^7
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
scripts/gpu_prof_f64.sh || exit 1
scripts/profile_cmd.sh f64x_1e7 python3 $R/scripts/run_f64x.py 10000000 20 > gpurun_out/prof_f64x_1e7.log 2>&1 || { tail -20 gpurun_out/prof_f64x_1e7.log; exit 1; }
python3 - <<'PY'
import json
d=json.load(open("gpurun_out/prof_f64x_1e7/summary.json"))
for k,v in d.items():
    print(k, {a: (round(b) if isinstance(b,float) else b) for a,b in v.items()})
PY
