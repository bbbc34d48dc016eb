#!/bin/bash
# Round-6 GPU session: GPU tests, smoke, the bench line (driver's 20 / 5 steps), calibrated
# traffic (tools/r06_traffic.sh), and a C5 parity-mode step split + kernel trace.
# Usage (gpurun): bash tools/r06_round.sh <tag> [skip-tests]
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -rf --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest_gpu exit $rc"; tail -5 $OUT/pytest_gpu.log
  [ $rc -eq 0 ] || exit 1
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; exit 1; }
fi
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail $OUT/bench.err; exit 1; }
echo bench ok
bash $R/tools/r06_traffic.sh $TAG/traffic > $OUT/traffic.log 2>&1 || { echo traffic failed; tail -20 $OUT/traffic.log; exit 1; }
echo traffic ok
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c5np -o trace -- python3 $R/tools/probe_np_c2.py --n 10000 --hyps 1000000 --outliers 0.6 --seed 5 --reps 2 --split > $OUT/c5np.json 2> $OUT/c5np.err || { echo c5 failed; exit 1; }
cat $OUT/c5np.json
