#!/bin/bash
# GPU tests + solve split (default vs RSAMD_SOLVE_DIAG=8: the Jacobi rank-2 path) + a short bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-quick}
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; st=$?
tail -3 $OUT/pytest_gpu.log
[ $st -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_gpu.log | head -20; exit 1; }
for d in 0 8; do
  echo -n "diag=$d " >> $OUT/solve_split.txt
  RSAMD_SOLVE_DIAG=$d timeout -k 10 120 python3 tools/solve_split.py >> $OUT/solve_split.txt 2>&1 || exit 1
done
cat $OUT/solve_split.txt
timeout -k 10 200 python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-extras > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('value',d['value'],'ms',d['ms_per_step'],'count',d['kernels_ms'],'parity',d.get('parity_mode',{}).get('value'))"
