#!/bin/bash
# round 4: the general (mixed) encoder at config 3, 10^7 records: timing, then trace + counters
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/enc1
timeout -k 10 200 python3 -u scripts/diag_encode.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/enc1/time.log || exit 1
scripts/profile_cmd.sh enc1 python3 $R/scripts/diag_encode.py > gpurun_out/enc1/prof.log 2>&1 || { tail gpurun_out/enc1/prof.log; exit 1; }
python3 - <<'PY'
import json
d=json.load(open("gpurun_out/prof_enc1/summary.json"))
for k,v in d.items():
    print(k, {a: (round(b) if isinstance(b,float) else b) for a,b in v.items()})
PY
