#!/bin/bash
# Kernel trace + stats of the C2 parse probe (product library).  Usage: bash tools/r05_prof_np.sh <tag>
set -o pipefail
TAG=${1:-r05pnp}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
NP_ONLY=2000 timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o np -- python3 $R/tools/np_kw_probe.py > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -5 $OUT/prof.log; exit 1; }
python3 $R/tools/kstats.py $OUT/prof/np_kernel_stats.csv
