#!/bin/bash
# rocprofv3 traces + counters of the f64 decoders at 10^8 and 10^7 (seq and run paths)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
scripts/profile_cmd.sh f64_1e8 python3 $R/scripts/prof_f64.py 100000000 9 seq run > gpurun_out/prof_f64_1e8.log 2>&1 || { tail -20 gpurun_out/prof_f64_1e8.log; exit 1; }
scripts/profile_cmd.sh f64_1e7 python3 $R/scripts/prof_f64.py 10000000 30 seq run > gpurun_out/prof_f64_1e7.log 2>&1 || { tail -20 gpurun_out/prof_f64_1e7.log; exit 1; }
for t in 1e8 1e7; do echo "== $t"; python3 - $t <<'PY'
import json,sys
d=json.load(open(f"gpurun_out/prof_f64_{sys.argv[1]}/summary.json"))
for k,v in d.items():
    print(k, {a: (round(b) if isinstance(b,float) else b) for a,b in v.items() if a in ("avg_ns","calls","FETCH_SIZE","WRITE_SIZE","SQ_WAIT_ANY","SQ_WAVE_CYCLES","SQ_BUSY_CYCLES","SQ_WAVES","SQ_INSTS_VALU","SQ_INSTS_SALU","SQ_ACTIVE_INST_ANY")})
PY
done
