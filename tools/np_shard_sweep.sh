#!/bin/bash
# Parity-stream layout sweep on one GPU: tools/probe_split.py (world 1) with rocprofv3 kernel
# stats per knob setting.  Usage (gpurun): bash tools/np_shard_sweep.sh <tag> c2|c5 "<env>" ...
set -o pipefail
TAG=$1; CASE=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$CASE" = c5 ]; then ARGS="--n 10000 --outliers 0.6 --seed 5 --hyps 1000000 --worlds 1 --reps 1"; else ARGS="--worlds 1 --reps 3"; fi
i=0
for e in "$@"; do
  i=$((i+1))
  ( cd /tmp && env $e timeout -k 10 250 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$CASE.$i -o np -- python3 $R/tools/probe_split.py $ARGS > $OUT/$CASE.$i.log 2>&1 ) || { echo "$e failed"; tail -3 $OUT/$CASE.$i.log; exit 1; }
  echo "== $CASE [$e]"; grep '^{"n"' $OUT/$CASE.$i.log | cut -c1-260
  python3 $R/tools/kstats.py $OUT/$CASE.$i/np_kernel_stats.csv > $OUT/$CASE.$i.kstats.txt
  sed -n 1,9p $OUT/$CASE.$i.kstats.txt
done
