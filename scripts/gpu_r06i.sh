#!/bin/bash
# round 6: general encoder A/B (3 rows per thread), counters of the final mixed decoder, bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_fullsize.py -k "encode or mixed" tests/test_gpu_archive.py > gpurun_out/r06i_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r06i_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for v in base g3 g3o5; do
  lib=$R/netidx_amd/build_ab/$v/libnxg_codec.so; [ $v = base ] && lib=$R/netidx_amd/lib/libnxg_codec.so
  NXG_LIB=$lib timeout -k 10 200 python3 -u scripts/ab_enc_mixed.py $v 2>&1 | grep -v amdgpu.ids || exit 1
done; done
bash scripts/profile_cmd.sh r06_mixed_final python3 $R/scripts/ab_mixed.py plainonly > gpurun_out/r06i_mixed_prof.log 2>&1 || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/prof_r06_mixed_final/summary.json'))
for k,v in d.items():
  if 'fmx' in k: print(k, round(v['avg_ns']/1e3,1), 'us VALU', v.get('SQ_INSTS_VALU'), 'LDSconf', v.get('SQ_LDS_BANK_CONFLICT'), 'LDSact', v.get('SQ_ACTIVE_INST_LDS'), 'FETCH', v.get('FETCH_SIZE'), 'WRITE', v.get('WRITE_SIZE'))"
timeout -k 10 600 python -u bench.py > gpurun_out/r06i_bench.json 2> gpurun_out/r06i_bench.err
rc=$?; cut -c1-200 gpurun_out/r06i_bench.json; exit $rc
