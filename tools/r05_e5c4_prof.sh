#!/bin/bash
# Kernel traces of the five-point E-RANSAC extra (C2 shape) and the C4 ring (tools/probe_*.py).
# Usage (through gpurun): bash tools/r05_e5c4_prof.sh <tag>
set -o pipefail
TAG=${1:-r05ec}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 200 python3 $R/tools/probe_e5.py > $OUT/e5.txt 2>&1 || { echo "e5 probe failed"; tail -5 $OUT/e5.txt; exit 1; }
cat $OUT/e5.txt
timeout -k 10 200 python3 $R/tools/probe_c4.py > $OUT/c4.txt 2>&1 || { echo "c4 probe failed"; tail -5 $OUT/c4.txt; exit 1; }
cat $OUT/c4.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_e5 -o e5 -- python3 $R/tools/probe_e5.py > $OUT/prof_e5.log 2>&1 || { echo "rocprof e5 failed"; tail -5 $OUT/prof_e5.log; exit 1; }
echo "== e5"; python3 $R/tools/kstats.py $(find $OUT/prof_e5 -name "*kernel_stats.csv")
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o c4 -- python3 $R/tools/probe_c4.py > $OUT/prof_c4.log 2>&1 || { echo "rocprof c4 failed"; tail -5 $OUT/prof_c4.log; exit 1; }
echo "== c4"; python3 $R/tools/kstats.py $(find $OUT/prof_c4 -name "*kernel_stats.csv")
