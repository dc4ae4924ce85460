#!/bin/bash
# PMC passes over the standalone f64 probe: LDS bank conflicts and the instruction mix of the
# single-pass decoder (one pass per counter group; each pass under its own time limit).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=${N:-100000000}
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
rm -rf $R/gpurun_out/pmc_lds1 $R/gpurun_out/pmc_lds2
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_BUSY_CYCLES --output-format csv -d $R/gpurun_out/pmc_lds1 -o run -- $R/scripts/probe_f64 $N 3 > $R/gpurun_out/pmc_lds1.log 2>&1 || { tail -5 $R/gpurun_out/pmc_lds1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM --output-format csv -d $R/gpurun_out/pmc_lds2 -o run -- $R/scripts/probe_f64 $N 3 > $R/gpurun_out/pmc_lds2.log 2>&1 || { tail -5 $R/gpurun_out/pmc_lds2.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections, os
R = os.environ.get("GRAFT_REPO_ROOT", ".")
for d in ("pmc_lds1", "pmc_lds2"):
    f = glob.glob(f"{R}/gpurun_out/{d}/**/*counter_collection.csv", recursive=True)
    if not f:
        print(d, "no csv"); continue
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"][:40]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[(k, r["Counter_Name"])] += 1
    for k, cs in acc.items():
        if "1p" not in k and "stream" not in k: continue
        calls = max(n[(k, c)] for c in cs)
        print(d, k, {c: "%.4g" % (v / calls) for c, v in cs.items()})
PY
