#!/bin/bash
# round 6: rocprofv3 evidence -- the mixed decoder (this round's build and the round-5 variant),
# the random-order f64 decoder, the sequential-id f64 encoder's writing launches alone
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/profile_cmd.sh r06_mixed python3 $R/scripts/ab_mixed.py plainonly > gpurun_out/r06d_mixed.log 2>&1
rc=$?; tail -40 gpurun_out/r06d_mixed.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
NXG_LIB=$R/netidx_amd/build_ab/old/libnxg_codec.so bash scripts/profile_cmd.sh r06_mixed_old python3 $R/scripts/ab_mixed.py plainonly > gpurun_out/r06d_mixed_old.log 2>&1
rc=$?; tail -40 gpurun_out/r06d_mixed_old.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
AB_ENC_PATHS=seq bash scripts/profile_cmd.sh r06_enc_seq python3 $R/scripts/ab_enc_f64.py prof 10000000 100000000 > gpurun_out/r06d_enc.log 2>&1
rc=$?; tail -30 gpurun_out/r06d_enc.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
bash scripts/profile_cmd.sh r06_f64x python3 $R/scripts/ab_f64x.py prof 10000000 > gpurun_out/r06d_f64x.log 2>&1
rc=$?; tail -30 gpurun_out/r06d_f64x.log | cut -c1-200; exit $rc
