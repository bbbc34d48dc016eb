#!/bin/bash
# C4 ring: the fused device call (rs_pairs_two_view) against the separate calls, interleaved,
# then the fused path's kernel trace.  Usage (through gpurun): bash tools/r05_c4_fused.sh <tag>
set -o pipefail
TAG=${1:-r05c4f}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for pass in 1 2 3; do
  echo "fused pass $pass $(timeout -k 10 100 python3 $R/tools/probe_c4.py)" || exit 1
  echo "separate pass $pass $(PROBE_UNFUSED=1 timeout -k 10 100 python3 $R/tools/probe_c4.py)" || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_fused -o c4 -- python3 $R/tools/probe_c4.py > $OUT/prof_fused.log 2>&1 || { echo "rocprof failed"; exit 1; }
echo "== fused"; python3 $R/tools/kstats.py $(find $OUT/prof_fused -name "*kernel_stats.csv") > $OUT/kstats_fused.txt; sed -n 1,13p $OUT/kstats_fused.txt
