#!/bin/bash
# GPU tests + 1-GPU bench + a 2-rank bench rehearsal on one GPU (gloo record exchange).
set -o pipefail
TAG=${1:-chk}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
st=$?; echo "pytest_gpu exit $st" >> $OUT/pytest_gpu.log; tail -3 $OUT/pytest_gpu.log
[ $st -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 400 python bench.py --steps 100 --warmup 200 > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'], d['roofline']['frac'], d.get('fp64_count',{}).get('value'), d['parity_mode'])"
if [ -n "$TWO" ]; then
RSAMD_BENCH_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 20 --no-extras --no-cpu-baseline > $OUT/bench2.json 2> $OUT/bench2.err || { echo bench2 failed; tail $OUT/bench2.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench2.json'));print(d['value'], d['config']['exchange'], d['parity_mode'])"
fi
