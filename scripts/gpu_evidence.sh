set -o pipefail
mkdir -p gpurun_out
timeout -k 5 120 ./scripts/probe_f64 100000000 20 > gpurun_out/probe_1e8.log 2>&1 && \
timeout -k 5 60 ./scripts/probe_f64 10000000 20 > gpurun_out/probe_1e7.log 2>&1 && \
timeout -k 5 120 ./scripts/probe_copy 100000000 > gpurun_out/copy_1e8.log 2>&1 && \
timeout -k 5 60 ./scripts/probe_copy 10000000 > gpurun_out/copy_1e7.log 2>&1 && \
bash scripts/gpu_round.sh
