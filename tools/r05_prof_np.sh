#!/bin/bash
# Kernel trace + stats of the C2 parse probe, the product library and lib_ab variants.
# Usage (through gpurun): bash tools/r05_prof_np.sh <tag> [ab-lib ...]
set -o pipefail
TAG=${1:-r05pnp}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for v in prod "$@"; do
  if [ $v = prod ]; then unset RSAMD_LIB; else export RSAMD_LIB=$R/tsbb15-3d-reconstruction-project_amd/lib_ab/$v/librsamd.so; fi
  NP_ONLY=2000 timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$v -o np -- python3 $R/tools/np_kw_probe.py > $OUT/prof_$v.log 2>&1 || { echo "rocprof $v failed"; tail -5 $OUT/prof_$v.log; exit 1; }
  echo "== $v"
  python3 $R/tools/kstats.py $OUT/prof_$v/np_kernel_stats.csv
done
