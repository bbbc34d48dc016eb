#!/bin/bash
# Round 4: the projection test, bench.py's own 2-rank launcher on one GPU (both ranks on
# device 0: RCCL refuses that, so the exchange falls back to the TCP hub), and a full 1-GPU
# bench line with parity_mode.split_projection.
# Usage (through gpurun): bash tools/r04_launch.sh <tag>
set -o pipefail
TAG=${1:-r04a}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_np_shard.py -x -q -k projection --timeout 120 --timeout-method thread > $OUT/pytest_proj.log 2>&1 || { echo projection test failed; tail -30 $OUT/pytest_proj.log; exit 1; }
tail -3 $OUT/pytest_proj.log
RSAMD_BENCH_DEVICE=0 timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 50 > $OUT/bench2.json 2> $OUT/bench2.err || { echo bench2 failed; tail -30 $OUT/bench2.err; exit 1; }
python -c "import json,sys; d=json.load(open('$OUT/bench2.json')); print('n_gpus', d['n_gpus'], d['config']['exchange'], d['value'])"
timeout -k 10 500 python bench.py --steps 100 --warmup 200 > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -30 $OUT/bench.err; exit 1; }
python - <<EOF
import json
d = json.load(open("$OUT/bench.json"))
print("value", d["value"], "parity ms", d["parity_mode"]["ms"])
for W, r in d["parity_mode"]["split_projection"]["worlds"].items():
    print(W, round(r["projected_ms"], 3), round(r["strong_scaling_efficiency"], 3), r["winner_equals_serial"], {k: [round(x, 3) for x in v] for k, v in r["per_rank_ms"].items()})
print(json.dumps(d["extras"].get("c5_parity")))
print(json.dumps(d["extras"].get("getFFromLabCode_dino_noisy")))
EOF
