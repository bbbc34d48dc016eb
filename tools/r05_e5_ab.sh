#!/bin/bash
# E5 A/B: tools/probe_e5.py on the product and lib_ab variants, interleaved three times.
# Usage (through gpurun): bash tools/r05_e5_ab.sh <variant...>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp
for pass in 1 2 3; do
  for v in prod "$@"; do
    if [ $v = prod ]; then unset RSAMD_LIB; else export RSAMD_LIB=$R/tsbb15-3d-reconstruction-project_amd/lib_ab/$v/librsamd.so; fi
    echo "$v pass $pass $(timeout -k 10 100 python3 $R/tools/probe_e5.py)" || exit 1
  done
done
