#!/bin/bash
# f64 probe only (A/B variants), 10^8 then 10^7 records.
set -o pipefail
mkdir -p gpurun_out
timeout -k 5 120 ./scripts/probe_f64 100000000 20 > gpurun_out/probe_1e8.log 2>&1; rc=$?
grep -v cycles gpurun_out/probe_1e8.log | head -24; [ $rc -eq 0 ] || exit $rc
timeout -k 5 60 ./scripts/probe_f64 10000000 20 > gpurun_out/probe_1e7.log 2>&1; rc=$?
head -18 gpurun_out/probe_1e7.log; exit $rc
