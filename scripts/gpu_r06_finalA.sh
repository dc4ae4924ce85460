#!/bin/bash
# round 6 last (A): the whole GPU suite, smoke(), the default bench line, and the bench as the
# driver runs it (--steps 20 --warmup 5)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
T=${TAG:-r06z}
TAG=$T scripts/gpu_r04b.sh || exit 1
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$T/bench_driver_cmd.json 2> gpurun_out/$T/bench_driver_cmd.err || { tail -20 gpurun_out/$T/bench_driver_cmd.err; exit 1; }
tail -c 600 gpurun_out/$T/bench_driver_cmd.json
