#!/bin/bash
# Kernel trace of the f64 decode bench at 10^7 and 10^8 (probe + emit split), TAG names the dir.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-t}
export TMPDIR=/tmp
cd /tmp
for N in 10000000 100000000; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/tr_${TAG}_$N -o tr -- python3 $R/bench.py --steps 40 --warmup 3 --no-extras --cpu-seconds 0.2 --records $N > $R/gpurun_out/tr_${TAG}_$N.json 2> $R/gpurun_out/tr_${TAG}_$N.err || exit 1
done
cd $R && python3 - "$TAG" <<'PY'
import csv, glob, json, sys
tag = sys.argv[1]
for n in ("10000000", "100000000"):
    f = glob.glob(f"gpurun_out/tr_{tag}_{n}/**/*kernel_stats.csv", recursive=True)[0]
    rows = {r["Name"].split("(")[0]: float(r["AverageNs"]) for r in csv.DictReader(open(f))}
    b = json.loads(open(f"gpurun_out/tr_{tag}_{n}.json").read().strip().splitlines()[-1])
    print(n, {k: round(v / 1e3, 2) for k, v in rows.items() if "f64r" in k}, "bench ms", b["ms_per_step"], "frac", b["roofline"]["frac"])
PY
