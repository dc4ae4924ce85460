#!/bin/bash
# round 4: fast mixed decoder A/B -- lean count (adaptive, default) vs full count
# (NXG_FMX_COUNT=full), lean emit rounds on / off -- then the trace + counters of the default
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/mix1
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mixed_fast.py tests/test_gpu_dispatch.py tests/test_gpu_multi.py > gpurun_out/mix1/tests.log 2>&1 || { tail -30 gpurun_out/mix1/tests.log; exit 1; }
tail -2 gpurun_out/mix1/tests.log
for rep in 1 2; do
  for v in base fullcount lean; do
    lib=$R/netidx_amd/lib/libnxg_codec.so
    env=""
    case $v in
      fullcount) env="NXG_FMX_COUNT=full";;
      lean) env="NXG_FMX_COUNT=lean";;
    esac
    env $env NXG_LIB=$lib timeout -k 10 300 python3 -u scripts/ab_mixed.py $v 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/mix1/ab.log || exit 1
  done
done
scripts/profile_cmd.sh mix1 python3 $R/scripts/ab_mixed.py trace > gpurun_out/mix1/prof.log 2>&1 || { tail gpurun_out/mix1/prof.log; exit 1; }
python3 - <<'PY'
import json
d=json.load(open("gpurun_out/prof_mix1/summary.json"))
for k,v in d.items():
    print(k, {a: (round(b) if isinstance(b,float) else b) for a,b in v.items() if a in ("avg_ns","calls","SQ_INSTS_VALU","SQ_INSTS_SALU","SQ_WAVES","SQ_INSTS_LDS","SQ_LDS_BANK_CONFLICT","SQ_ACTIVE_INST_LDS","SQ_WAIT_ANY","SQ_WAVE_CYCLES")})
PY
