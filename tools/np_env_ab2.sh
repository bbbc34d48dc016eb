#!/bin/bash
# C2 parse kernel stats per environment setting (same library), interleaved.
# Usage (gpurun): bash tools/np_env_ab2.sh <tag> "VAR=a" "VAR=b" ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-envab}; shift
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
n=0
for v in "$@"; do
  n=$((n+1))
  env $v NP_ONLY=2000 timeout -k 5 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/v$n -o np -- python3 $R/tools/np_kw_probe.py > $OUT/v$n.log 2>&1 || { echo "$v failed"; tail -3 $OUT/v$n.log; exit 1; }
  echo "$v $(grep gpu_ms $OUT/v$n.log | cut -c1-110)"
  python3 $R/tools/kstats.py $OUT/v$n/np_kernel_stats.csv | grep -E "tuples|track|entry"
done
