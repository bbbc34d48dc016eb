#!/bin/bash
# Counting-kernel launch-shape sweep: the wave timeline (RSAMD_TSTAMP) of the default launch,
# then the headline bench's HIP-event kernel time per setting (arguments like RSAMD_QCHUNK=64
# or RSAMD_WAVES=4096; "-" is the default).
set -o pipefail
TAG=${1:-csw}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
RSAMD_TSTAMP=/tmp/ts_$$.bin timeout -k 10 120 python tools/count_timeline.py > $OUT/timeline.txt 2>&1 || { echo timeline failed; tail $OUT/timeline.txt; exit 1; }
cat $OUT/timeline.txt
i=0
for kv in "$@"; do
  i=$((i+1))
  if [ "$kv" = "-" ]; then envs=""; else envs="$kv"; fi
  env $envs timeout -k 10 300 python bench.py --steps 200 --warmup 200 --no-extras --no-parity-mode --no-cpu-baseline --no-fp64-count > $OUT/bench_$i.json 2> $OUT/bench_$i.err || { echo "bench $kv failed"; tail $OUT/bench_$i.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_$i.json'));print('$kv', d['value'], d['roofline']['per_launch']['avg_ms'])"
done
