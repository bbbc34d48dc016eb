#!/bin/bash
# Round-4 GPU session: all GPU tests, the two timelines (counting kernel waves, parse chunks),
# then a full 1-GPU bench line.  Usage (through gpurun): bash tools/r04_round.sh <tag>
set -o pipefail
TAG=${1:-r04b}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
st=$?
tail -4 $OUT/pytest_gpu.log
[ $st -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_gpu.log | head -20; exit 1; }
RSAMD_TSTAMP=/tmp/cts.bin timeout -k 10 200 python tools/count_timeline.py > $OUT/count_timeline.txt 2>&1 || { echo count timeline failed; tail $OUT/count_timeline.txt; exit 1; }
cat $OUT/count_timeline.txt
timeout -k 10 200 python tools/np_timeline.py 10000 20000 3 > $OUT/np_timeline_n10k.json 2> $OUT/np_timeline.err || { echo timeline failed; tail $OUT/np_timeline.err; exit 1; }
bash tools/e5_split_ab.sh $TAG/e5 || exit 1
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
python - <<PY
import json
d = json.load(open("$OUT/bench.json"))
print("value", d["value"], "ms", d["ms_per_step"], "frac", d["roofline"]["frac"], "parity ms", d["parity_mode"]["ms"])
print(json.dumps(d["cpu_baseline"]["reference_loop"])[:400])
PY
