#!/bin/bash
# Counting-kernel slice schedule A/B (RSAMD_QSCHED: 0 = equal slices, p > 0 = decreasing), headline
# bench per value, interleaved twice; then the C2 GPU tests under the last value.
set -o pipefail
TAG=${1:-qs}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for rep in 1 2; do
for v in "$@"; do
  RSAMD_QSCHED=$v timeout -k 10 200 python bench.py --steps 200 --warmup 200 --no-extras --no-parity-mode --no-cpu-baseline --no-fp64-count > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { echo "bench $v failed"; tail $OUT/bench_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_$v.json'));print('$v', d['value'], d['roofline']['per_launch']['avg_ms'], d['roofline']['frac'])"
done
done
RSAMD_QSCHED=${@: -1} timeout -k 10 300 python -u -m pytest tests/test_gpu_f8.py tests/test_gpu_full_parity.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
st=$?; tail -2 $OUT/pytest.log; exit $st
