#!/bin/bash
# round 5: archive entry-guess A/B (PRE bytes walked before a tile, fix passes), encoder A/B
# (OR staging) and phase stamps, and the dispatch split; each GPU step under its own limit
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
VARIANTS="eor" scripts/gpu_enc2.sh || exit 1
for v in encp eorp; do
  echo "== stamps $v"
  NXG_LIB=$R/netidx_amd/build_ab/$v/libnxg_codec.so timeout -k 10 120 python3 scripts/stamps_enc.py 10000000 2>&1 | grep -v amdgpu.ids || exit 1
done
scripts/gpu_ab_arch2.sh base pre192 pre256 pre256f1 || exit 1
scripts/gpu_disp_prof.sh || exit 1
