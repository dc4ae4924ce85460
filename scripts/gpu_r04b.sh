#!/bin/bash
# round 4: the whole GPU suite, smoke(), then the default bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/${TAG:-r04b}
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/${TAG:-r04b}/tests.log 2>&1 || { tail -40 gpurun_out/${TAG:-r04b}/tests.log; exit 1; }
tail -3 gpurun_out/${TAG:-r04b}/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG:-r04b}/smoke.log 2>&1 || { tail -20 gpurun_out/${TAG:-r04b}/smoke.log; exit 1; }
tail -1 gpurun_out/${TAG:-r04b}/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG:-r04b}/bench.json 2> gpurun_out/${TAG:-r04b}/bench.err || { tail -20 gpurun_out/${TAG:-r04b}/bench.err; exit 1; }
tail -c 3000 gpurun_out/${TAG:-r04b}/bench.json
