#!/bin/bash
# round 4: the fast mixed decoder on the config-3 frame with Heartbeats and long strings only:
# trace + counters, and the per-call recount diagnostics
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/mix2
scripts/profile_cmd.sh mix2 python3 $R/scripts/ab_mixed.py ctlonly > gpurun_out/mix2/prof.log 2>&1 || { tail gpurun_out/mix2/prof.log; exit 1; }
grep ctlonly gpurun_out/mix2/prof.log | head -2
python3 - <<'PY'
import json
d=json.load(open("gpurun_out/prof_mix2/summary.json"))
for k,v in d.items():
    print(k, {a: (round(b) if isinstance(b,float) else b) for a,b in v.items() if a in ("avg_ns","calls","SQ_INSTS_VALU","SQ_INSTS_SALU","SQ_WAVES","SQ_INSTS_LDS","SQ_LDS_BANK_CONFLICT","SQ_ACTIVE_INST_LDS","SQ_WAIT_ANY","SQ_WAVE_CYCLES","FETCH_SIZE","WRITE_SIZE")})
PY
