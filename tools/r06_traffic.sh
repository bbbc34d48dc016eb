#!/bin/bash
# Calibrated HBM traffic: FETCH_SIZE / WRITE_SIZE per access shape on known
# bytes (tools/ubench/fetch_calib), then the counting kernel (C2 bench launches) and the parse
# kernels (C2 parity runs), one counter block per rocprofv3 pass.
# Usage (gpurun): bash tools/r06_traffic.sh <tag>
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
CAL=$R/tools/ubench/fetch_calib
timeout -s KILL 120 $CAL > $OUT/cal.json || { echo "calib run failed"; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/cal_$c -o pmc -- $CAL > $OUT/cal_$c.log 2>&1 || { echo "calib pmc $c failed"; exit 1; }
done
B="python3 $R/bench.py --steps 50 --warmup 200 --no-cpu-baseline --no-parity-mode --no-extras --no-fp64-count"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $OUT/count_$c -o pmc -- $B > $OUT/count_$c.log 2>&1 || { echo "count pmc $c failed"; exit 1; }
done
P="python3 $R/tools/probe_np_c2.py --reps 4"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $OUT/parse_$c -o pmc -- $P > $OUT/parse_$c.log 2>&1 || { echo "parse pmc $c failed"; exit 1; }
done
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/parse_trace -o trace -- $P --split > $OUT/parse_trace.log 2>&1 || { echo "parse trace failed"; exit 1; }
python3 $R/tools/traffic_summary.py $OUT > $OUT/traffic.json && cat $OUT/traffic.json
