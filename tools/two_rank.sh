#!/bin/bash
# 2-rank bench rehearsal on a one-GPU box (both ranks on device 0: RCCL refuses two ranks on
# one GPU, so the record exchange falls back to gloo; the data path is the same per rank).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-two}
mkdir -p $OUT
cd $R
RSAMD_BENCH_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 20 > $OUT/bench2.json 2> $OUT/bench2.err
st=$?
echo "rc=$st"
[ $st -eq 0 ] || { tail -5 $OUT/bench2.err; exit 1; }
python3 - "$OUT/bench2.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(d["value"], d["n_gpus"], d["config"]["exchange"])
print(json.dumps(d["parity_mode"])[:400])
print(sorted(d.get("extras", {}).keys()))
PY
