#!/bin/bash
# Five-point solver check: GPU known-answer tests, then the bench's e5 extra.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-e5}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_essential.py tests/test_oracle_essential.py -q -x --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
st=$?; tail -3 $OUT/pytest.log; [ $st -eq 0 ] || exit 1
timeout -k 10 400 python bench.py --steps 20 --warmup 20 --no-parity-mode --no-cpu-baseline --no-fp64-count > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['extras']['e5_ransac_c2'])" $OUT/bench.json
