#!/bin/bash
# round 5: a clean trace of the north-star kernel -- the bench's 10^8 leg alone (every dispatch a
# full sequential-id decode), with FETCH / WRITE / SQ counters in their own passes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 120 python3 scripts/prof_f64_1e8.py 12 2 > gpurun_out/r05_1e8_plain.log 2>&1 || { cat gpurun_out/r05_1e8_plain.log; exit 1; }
cat gpurun_out/r05_1e8_plain.log
scripts/profile_cmd.sh r05_f64_1e8 python3 $R/scripts/prof_f64_1e8.py 12 2 > gpurun_out/r05_1e8_prof.log 2>&1 || { tail -20 gpurun_out/r05_1e8_prof.log; exit 1; }
python3 scripts/kdisp.py gpurun_out/prof_r05_f64_1e8/trace nxg_f64s --json gpurun_out/prof_r05_f64_1e8/dispatches.json
cat gpurun_out/prof_r05_f64_1e8/trace.log | grep "10^8"
