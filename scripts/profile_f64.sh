#!/bin/bash
# rocprofv3 evidence for the f64 decode bench line (run on the GPU box, from the repo root):
#   1. --kernel-trace --stats        per-kernel durations (must agree with bench.py's kernel_ms)
#   2. --pmc FETCH_SIZE / WRITE_SIZE HBM-side bytes, one counter per pass (no trace domains)
#   3. --pmc SQ_*                    wave-state / instruction-mix counters
# then scripts/summarize_profile.py writes profiles/<tag>_* and profiles/pmc_dec_f64.json.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
export TMPDIR=/tmp
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp
ARGS="--steps 20 --warmup 3 --no-extras --cpu-seconds 0.2 --records ${RECORDS:-10000000}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $R/bench.py $ARGS > $OUT/trace_bench.json 2> $OUT/trace.err \
 && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- python3 $R/bench.py $ARGS > $OUT/fetch_bench.json 2> $OUT/fetch.err \
 && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- python3 $R/bench.py $ARGS > $OUT/write_bench.json 2> $OUT/write.err \
 && timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $OUT/sq -o sq -- python3 $R/bench.py $ARGS > $OUT/sq_bench.json 2> $OUT/sq.err \
 && cd $R && python3 scripts/summarize_profile.py $OUT $TAG
