#!/bin/bash
# Overlap mode A/B: the GPU tests with RSAMD_OVERLAP=1, then the C2 bench line with RSAMD_OVERLAP=1 and 0 (the default).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-ovl}
mkdir -p $OUT
cd $R
RSAMD_OVERLAP=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
st=$?; tail -2 $OUT/pytest.log; [ $st -eq 0 ] || exit 1
for pass in 1 2; do
  for o in 1 0; do
    RSAMD_OVERLAP=$o timeout -k 10 300 python bench.py --steps 200 --warmup 200 --no-parity-mode --no-cpu-baseline --no-extras --no-fp64-count > $OUT/b$o.json 2> $OUT/b$o.err || { tail -5 $OUT/b$o.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['per_launch']['avg_ms'])" $OUT/b$o.json overlap=$o
  done
done
