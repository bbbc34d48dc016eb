#!/bin/bash
# Entry / tracking statistics of one C2 parse (diagnostic library, RSAMD_NP_STATS), default chunks.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r05npd}
mkdir -p $OUT
cd $R
rm -f $OUT/stats.bin
RSAMD_LIB=$R/tsbb15-3d-reconstruction-project_amd/lib_diag/librsamd.so RSAMD_NP_STATS=$OUT/stats.bin timeout -k 10 120 python3 tools/np_stats.py > $OUT/diag.log 2>&1 || { echo "diag failed"; tail $OUT/diag.log; exit 1; }
python3 tools/np_stats.py --read $OUT/stats.bin
