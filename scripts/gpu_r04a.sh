#!/bin/bash
# round 4: the new/changed GPU tests (sequential-id decoder, both f64 front ends, self-help
# look-backs), then the f64 decoders' traces and counters at 10^8 and 10^7
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/r04a
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_selfhelp.py tests/test_gpu_publish.py tests/test_gpu_archive.py tests/test_gpu_zstd.py tests/test_gpu_multi.py tests/test_gpu_multirank.py tests/test_gpu_f64_seq.py tests/test_gpu_api.py tests/test_gpu_fullsize.py > gpurun_out/r04a/tests.log 2>&1 || { tail -40 gpurun_out/r04a/tests.log; exit 1; }
tail -3 gpurun_out/r04a/tests.log
scripts/gpu_prof_f64.sh
