#!/bin/bash
# multi-GPU pieces on one GPU: range decode + link tests, 1-rank RCCL, then the N=2 rehearsal of
# bench.py over gloo with both ranks on cuda:0.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_api.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_multi.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed|Error" gpurun_out/pytest_multi.log | tail -25; [ $rc -eq 0 ] || exit $rc
BENCH_DIST_BACKEND=gloo BENCH_FORCE_DEVICE0=1 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 2 > gpurun_out/bench_n2_rehearsal.json 2> gpurun_out/bench_n2_rehearsal.err
rc=$?; cat gpurun_out/bench_n2_rehearsal.json; [ $rc -eq 0 ] || tail -20 gpurun_out/bench_n2_rehearsal.err; exit $rc
