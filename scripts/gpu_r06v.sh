#!/bin/bash
# round 6: the bench's kernel-time pass with and without the spin-kernel gate, --steps 20
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
for rep in 1 2; do for g in 500000 0; do
  BENCH_GATE_CYCLES=$g timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-extras --cpu-seconds 0.2 > gpurun_out/gate_$g.json 2> gpurun_out/gate_$g.err || { tail -20 gpurun_out/gate_$g.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/gate_$g.json').read().strip().splitlines()[-1])
print('gate $g rep $rep', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done; done
