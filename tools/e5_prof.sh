#!/bin/bash
# Kernel trace of the five-point E-RANSAC bench extra.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-e5p}
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o e5 -- python3 $R/tools/probe_e5.py > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -5 $OUT/prof.log; exit 1; }
python3 $R/tools/kstats.py $(find $OUT/prof -name "*kernel_stats.csv")
