#!/bin/bash
# Two-phase E5 root finder: C2 E-RANSAC time per RSAMD_E5_SPLIT (0 = one phase), two passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-e5s}
mkdir -p $OUT
cd $R
for pass in 1 2; do
  for sp in 0 5 6 8 10 12; do
    echo -n "split=$sp pass$pass " | tee -a $OUT/ab.txt
    RSAMD_E5_SPLIT=$sp timeout -k 10 120 python3 tools/probe_e5.py | tee -a $OUT/ab.txt || exit 1
  done
done
