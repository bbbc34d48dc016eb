#!/bin/bash
# Parity-stream check on the GPU: the probe (every tuple against the host replay, C2 and a
# C5-shaped stream), the parity-stream GPU tests, and a kernel trace of the C2 probe.
# Usage (through gpurun): bash tools/np_check.sh <tag>
set -o pipefail
TAG=${1:-npc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 200 python3 tools/np_kw_probe.py > $OUT/probe.jsonl 2> $OUT/probe.err || { echo "probe failed"; tail -5 $OUT/probe.err; exit 1; }
cat $OUT/probe.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_np_sampler.py tests/test_gpu_full_parity.py tests/test_gpu_np_shard.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
echo "pytest exit $?"; tail -3 $OUT/pytest.log
NP_ONLY=2000 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o np -- python3 tools/np_kw_probe.py > $OUT/prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
python3 tools/kstats.py $(find $OUT/prof -name "*kernel_stats.csv") || true
