#!/bin/bash
# Tracking statistics of the parity stream (diagnostic library build, lib_diag/).
set -o pipefail
TAG=${1:-npd}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for kw in ${KWS:-1048576}; do
  rm -f $OUT/stats_$kw.bin
  RSAMD_NP_KW=$kw RSAMD_LIB=$R/tsbb15-3d-reconstruction-project_amd/lib_diag/librsamd.so RSAMD_NP_STATS=$OUT/stats_$kw.bin timeout -k 10 120 python3 tools/np_stats.py > $OUT/diag_$kw.log 2>&1 || { echo "diag $kw failed"; tail $OUT/diag_$kw.log; exit 1; }
done
echo ok
