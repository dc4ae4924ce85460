#!/bin/bash
# rocprofv3 evidence for any program (run on the GPU box from the repo root):
#   scripts/profile_cmd.sh TAG python3 scripts/some_driver.py args...
# a kernel trace with stats, then FETCH_SIZE, WRITE_SIZE and two SQ counter groups, each pass its
# own run under its own time limit; per-kernel means per dispatch in gpurun_out/prof_$TAG/summary.json
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
export TMPDIR=/tmp
OUT=$R/gpurun_out/prof_$TAG
rm -rf $OUT
mkdir -p $OUT
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- "$@" > $OUT/trace.log 2>&1 \
 && timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- "$@" > $OUT/fetch.log 2>&1 \
 && timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- "$@" > $OUT/write.log 2>&1 \
 && timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES --output-format csv -d $OUT/sq1 -o run -- "$@" > $OUT/sq1.log 2>&1 \
 && timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH --output-format csv -d $OUT/sq2 -o run -- "$@" > $OUT/sq2.log 2>&1 \
 && cd $R && python3 scripts/summarize_pmc_dir.py $OUT
