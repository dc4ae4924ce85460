#!/bin/bash
# PMC pass over the standalone f64 probe (10^7 records): instruction mix and wait cycles.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
rm -rf $R/gpurun_out/pmc_f64
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH --output-format csv -d $R/gpurun_out/pmc_f64 -o run -- $R/scripts/probe_f64 10000000 3 > $R/gpurun_out/pmc_f64.log 2>&1
rc=$?; tail -2 $R/gpurun_out/pmc_f64.log; exit $rc
