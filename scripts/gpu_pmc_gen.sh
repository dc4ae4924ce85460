#!/bin/bash
# PMC passes over the general decode (config 3 at 1e7): instruction mix, LDS conflicts, waits.
# One counter group per pass, each under its own time limit; per-kernel means per dispatch.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
rm -rf $R/gpurun_out/pmc_gen1 $R/gpurun_out/pmc_gen2
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_BUSY_CYCLES --output-format csv -d $R/gpurun_out/pmc_gen1 -o run -- python3 $R/scripts/diag_general.py 10000000 > $R/gpurun_out/pmc_gen1.log 2>&1 || { tail -5 $R/gpurun_out/pmc_gen1.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d $R/gpurun_out/pmc_gen2 -o run -- python3 $R/scripts/diag_general.py 10000000 > $R/gpurun_out/pmc_gen2.log 2>&1 || { tail -5 $R/gpurun_out/pmc_gen2.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections, os
R = os.environ.get("GRAFT_REPO_ROOT", ".")
for d in ("pmc_gen1", "pmc_gen2"):
    f = glob.glob(f"{R}/gpurun_out/{d}/**/*counter_collection.csv", recursive=True)
    if not f:
        print(d, "no csv"); continue
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"].split("(")[0]
        if not k.startswith("nxg"): continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    for k, cs in acc.items():
        n = len(disp[k])
        print(d, k, n, {c: "%.4g" % (v / n) for c, v in sorted(cs.items())})
PY
