#!/bin/bash
# Interleaved A/B of five-point E-RANSAC library variants (lib_ab/<name>), two passes:
#   bash tools/e5_ab.sh <tag> <name>...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for pass in 1 2; do
  for n in "$@"; do
    echo -n "$n pass$pass "
    RSAMD_LIB=$R/tsbb15-3d-reconstruction-project_amd/lib_ab/$n/librsamd.so timeout -k 10 120 python3 tools/probe_e5.py | tee -a $OUT/ab.txt || exit 1
  done
done
