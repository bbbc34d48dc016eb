#!/bin/bash
# Parse timeline (product kernels' stamps) at C2 and N = 10 000, plus the sampler parity tests.
# Usage (through gpurun): bash tools/r04_np.sh <tag>
set -o pipefail
TAG=${1:-r04np}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_np_sampler.py tests/test_gpu_full_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_np.log 2>&1 || { echo np tests failed; tail -30 $OUT/pytest_np.log; exit 1; }
tail -2 $OUT/pytest_np.log
timeout -k 10 200 python tools/np_timeline.py 2000 100000 4 > $OUT/np_timeline_c2.json 2> $OUT/np_timeline.err || { echo timeline failed; tail $OUT/np_timeline.err; exit 1; }
cat $OUT/np_timeline_c2.json
timeout -k 10 200 python tools/np_timeline.py 10000 20000 3 > $OUT/np_timeline_n10k.json 2>> $OUT/np_timeline.err || { echo timeline2 failed; exit 1; }
timeout -k 10 200 python tools/np_kw_probe.py > $OUT/np_kw_probe.txt 2>&1 || echo "probe failed"
tail -5 $OUT/np_kw_probe.txt
