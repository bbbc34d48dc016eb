#!/bin/bash
# Parse A/B session: the parity tests, the C2 step split (probe_np_c2 --split, 8 runs) and
# optionally a C5 kernel trace + split.  Usage (gpurun): bash tools/r06_np.sh <tag> [c5] [notest]
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
if [ "$3" != "notest" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_np_sampler.py tests/test_gpu_full_parity.py tests/test_gpu_np_shard.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
fi
for i in 1 2; do
  timeout -k 10 120 python3 tools/probe_np_c2.py --reps 8 --split > $OUT/c2_$i.json || { echo c2 probe failed; exit 1; }
  cat $OUT/c2_$i.json
done
if [ "$2" = "c5" ]; then
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c5np -o trace -- python3 $R/tools/probe_np_c2.py --n 10000 --hyps 1000000 --outliers 0.6 --seed 5 --reps 2 --split > $OUT/c5np.json 2> $OUT/c5np.err || { echo c5 failed; exit 1; }
  cat $OUT/c5np.json
fi
