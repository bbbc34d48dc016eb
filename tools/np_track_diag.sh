#!/bin/bash
# Per-chunk statistics of the parity-stream parse (diagnostic library, automatic layout).
# Usage (through gpurun): bash tools/np_track_diag.sh <tag> [N]
set -o pipefail
TAG=${1:-npt}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
rm -f $OUT/stats.bin
NP_N=${2:-2000} RSAMD_LIB=$R/tsbb15-3d-reconstruction-project_amd/lib_diag/librsamd.so RSAMD_NP_STATS=$OUT/stats.bin timeout -k 10 120 python3 tools/np_stats.py > $OUT/run.log 2>&1 || { echo "diag failed"; tail $OUT/run.log; exit 1; }
python3 tools/np_stats.py --read $OUT/stats.bin
