#!/bin/bash
# Parity-stream session: sampler tests, timing probe, rocprofv3 kernel stats of the probe.
# Usage (through gpurun): bash tools/np_round.sh <tag> [extra env assignments...]
set -o pipefail
TAG=${1:-np}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_np_sampler.py tests/test_gpu_full_parity.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
st=$?
echo "pytest exit $st" >> $OUT/pytest.log
tail -3 $OUT/pytest.log
[ $st -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/probe_np_sampler.py > $OUT/probe.jsonl 2> $OUT/probe.err || { echo probe failed; tail $OUT/probe.err; exit 1; }
cat $OUT/probe.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o np -- python3 tools/probe_np_sampler.py > $OUT/prof.log 2>&1 || { echo rocprof failed; exit 1; }
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 $f | head -20
