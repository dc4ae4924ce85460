#!/bin/bash
# Instruction-mix counters for the f64 decode kernels via the standalone probe (one --pmc pass
# per counter group; no trace domains combined with --pmc).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=$R/gpurun_out/pmc
mkdir -p $OUT
cd /tmp
N=${1:-10000000}
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $OUT/a -o a -- $R/scripts/probe_f64 $N 1 > $OUT/a.log 2>&1 \
 && timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/b -o b -- $R/scripts/probe_f64 $N 1 > $OUT/b.log 2>&1 \
 && timeout -k 10 200 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM --output-format csv -d $OUT/c -o c -- $R/scripts/probe_f64 $N 1 > $OUT/c.log 2>&1
