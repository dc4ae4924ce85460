#!/bin/bash
# rocprofv3 kernel trace + HBM counters (separate --pmc passes) for the f64 decode bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=$R/gpurun_out/prof
mkdir -p $OUT
cd /tmp
ARGS="--steps 20 --warmup 3 --no-extras --cpu-seconds 0.2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $R/bench.py $ARGS > $OUT/trace_bench.json 2> $OUT/trace.err \
 && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- python3 $R/bench.py $ARGS > $OUT/fetch_bench.json 2> $OUT/fetch.err \
 && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- python3 $R/bench.py $ARGS > $OUT/write_bench.json 2> $OUT/write.err \
 && timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o sq -- python3 $R/bench.py $ARGS > $OUT/sq_bench.json 2> $OUT/sq.err
