#!/bin/bash
# Counting-kernel A/B: GPU tests of the RANSAC-F path, then the headline bench per RSAMD_COUNT
# value (HIP-event kernel time in roofline.per_launch.avg_ms), then rocprofv3 kernel stats.
set -o pipefail
TAG=${1:-cab}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_f8.py tests/test_gpu_full_parity.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
st=$?; echo "pytest exit $st" >> $OUT/pytest.log; tail -2 $OUT/pytest.log
[ $st -eq 0 ] || exit 1
for v in "$@"; do
  RSAMD_COUNT=$v timeout -k 10 300 python bench.py --steps 200 --warmup 200 --no-extras --no-parity-mode --no-cpu-baseline --no-fp64-count > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { echo "bench $v failed"; tail $OUT/bench_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_$v.json'));print('$v', d['value'], d['roofline']['per_launch']['avg_ms'], d['roofline']['frac'])"
done
RSAMD_COUNT=$1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o cnt -- python3 bench.py --steps 200 --warmup 200 --no-extras --no-parity-mode --no-cpu-baseline --no-fp64-count > $OUT/prof.log 2>&1 || { echo rocprof failed; exit 1; }
