#!/bin/bash
# Stall breakdown of the counting kernel on a warmed bench: wait / issue counters and the
# scalar data cache (one rocprofv3 --pmc pass per counter group).
set -o pipefail
TAG=${1:-cpm2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
rocprofv3 -L > $OUT/avail.txt 2>&1 || true
grep -oE "\b(SQC|SQ)_[A-Z0-9_]+" $OUT/avail.txt | sort -u > $OUT/names.txt || true
B="python3 bench.py --steps 50 --warmup 200 --no-extras --no-parity-mode --no-cpu-baseline --no-fp64-count"
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o pmc -- $B > $OUT/p$i.log 2>&1 || echo "pass $i ($grp) failed"
done
python3 tools/pmc_read.py $OUT k_f8_count32q
