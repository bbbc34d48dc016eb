#!/bin/bash
# C4 ring A/B: tools/probe_c4.py on the product and lib_ab variants, interleaved twice, then the
# product's kernel trace.  Usage (through gpurun): bash tools/r05_c4_ab.sh <tag> <variant...>
set -o pipefail
TAG=${1:-r05c4}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for pass in 1 2; do
  for v in prod "$@"; do
    if [ $v = prod ]; then unset RSAMD_LIB; else export RSAMD_LIB=$R/tsbb15-3d-reconstruction-project_amd/lib_ab/$v/librsamd.so; fi
    echo "$v pass $pass $(timeout -k 10 100 python3 $R/tools/probe_c4.py)" || exit 1
  done
done
unset RSAMD_LIB
for v in prod "$@"; do
  if [ $v = prod ]; then unset RSAMD_LIB; else export RSAMD_LIB=$R/tsbb15-3d-reconstruction-project_amd/lib_ab/$v/librsamd.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$v -o c4 -- python3 $R/tools/probe_c4.py > $OUT/prof_$v.log 2>&1 || { echo "rocprof failed"; exit 1; }
  echo "== $v"; python3 $R/tools/kstats.py $(find $OUT/prof_$v -name "*kernel_stats.csv") > $OUT/kstats_$v.txt; sed -n 1,9p $OUT/kstats_$v.txt
done
