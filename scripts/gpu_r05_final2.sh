#!/bin/bash
# round 5 last: the whole GPU suite, smoke(), the default bench line, and the N=2 rehearsal of
# bench.py (gloo, both ranks on cuda:0: the multi-rank legs run, their times are no scaling data)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
TAG=${TAG:-r05y} scripts/gpu_r04b.sh || exit 1
BENCH_DIST_BACKEND=gloo BENCH_FORCE_DEVICE0=1 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 2 > gpurun_out/${TAG:-r05y}/bench_n2_rehearsal.json 2> gpurun_out/${TAG:-r05y}/bench_n2_rehearsal.err
rc=$?; tail -c 1500 gpurun_out/${TAG:-r05y}/bench_n2_rehearsal.json; [ $rc -eq 0 ] || tail -20 gpurun_out/${TAG:-r05y}/bench_n2_rehearsal.err; exit $rc
