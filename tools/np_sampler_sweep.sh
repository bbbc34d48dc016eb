#!/bin/bash
# Kernel-time breakdown of the GPU parity stream at several chunk lengths (RSAMD_NP_KW).
# Usage (through gpurun): bash tools/np_sampler_sweep.sh <tag> [kw ...]
TAG=${1:-np}
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
for KW in "${@:-262144}"; do
  export RSAMD_NP_KW=$KW
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kw$KW -o np -- python3 tools/probe_np_sampler.py > $OUT/kw$KW.log 2>&1 || { echo "kw $KW failed"; exit 1; }
  cat $OUT/kw$KW.log
done
