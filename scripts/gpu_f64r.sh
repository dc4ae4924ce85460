#!/bin/bash
# length-run f64 decode probe (scripts/probe_f64r.hip), 10^8 then 10^7 records.
set -o pipefail
mkdir -p gpurun_out
timeout -k 5 150 ./scripts/probe_f64r 100000000 20 > gpurun_out/probe_f64r_1e8.log 2>&1; rc=$?
cat gpurun_out/probe_f64r_1e8.log; [ $rc -eq 0 ] || exit $rc
timeout -k 5 90 ./scripts/probe_f64r 10000000 20 > gpurun_out/probe_f64r_1e7.log 2>&1; rc=$?
cat gpurun_out/probe_f64r_1e7.log; exit $rc
