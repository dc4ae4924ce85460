#!/bin/bash
# round 6 last (B): the N=2 rehearsal of bench.py (gloo, both ranks on cuda:0: the multi-rank legs
# run and are checked, their times are no scaling data), then a kernel trace of the bench command
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
T=${TAG:-r06z}
mkdir -p gpurun_out/$T
BENCH_DIST_BACKEND=gloo BENCH_FORCE_DEVICE0=1 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 2 > gpurun_out/$T/bench_n2_rehearsal.json 2> gpurun_out/$T/bench_n2_rehearsal.err || { tail -20 gpurun_out/$T/bench_n2_rehearsal.err; exit 1; }
tail -c 400 gpurun_out/$T/bench_n2_rehearsal.json
rm -rf gpurun_out/$T/bench_prof
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$T/bench_prof -o t -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $R/gpurun_out/$T/bench_prof.json 2> $R/gpurun_out/$T/bench_prof.err || { tail -20 $R/gpurun_out/$T/bench_prof.err; exit 1; }
cd $R
f=$(find gpurun_out/$T/bench_prof -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv
for r in list(csv.DictReader(open('$f')))[:14]:
    print(r['Name'].split('(')[0][:50], r['Calls'], round(float(r['AverageNs'])/1e3, 1))"
