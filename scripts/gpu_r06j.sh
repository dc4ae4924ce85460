#!/bin/bash
# round 6: order experiment (mixed decode after heavy load), partition counters
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u scripts/exp_order.py 2>&1 | grep -v amdgpu.ids || exit 1
bash scripts/profile_cmd.sh r06_part python3 $R/scripts/ab_partition.py prof > gpurun_out/r06j_part_prof.log 2>&1 || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/prof_r06_part/summary.json'))
for k,v in d.items():
  if 'part' in k: print(k, {x: v.get(x) for x in ('avg_ns','FETCH_SIZE','WRITE_SIZE','SQ_INSTS_VALU','SQ_INSTS_SALU','SQ_INSTS_LDS','SQ_WAIT_ANY','SQ_WAVE_CYCLES','SQ_ACTIVE_INST_ANY','SQ_LDS_BANK_CONFLICT')})"
