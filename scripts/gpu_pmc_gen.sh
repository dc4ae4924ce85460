#!/bin/bash
# PMC pass over the general decode (config 3 at 1e7): instruction mix and wait cycles.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_gen
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH --output-format csv -d gpurun_out/pmc_gen -o run -- python3 scripts/diag_general.py 10000000 > gpurun_out/pmc_gen.log 2>&1
rc=$?; tail -3 gpurun_out/pmc_gen.log; exit $rc
