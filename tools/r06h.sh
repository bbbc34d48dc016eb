#!/bin/bash
# GPU tests + smoke, the C2 tuple-workgroup A/B, then the bench line (driver settings).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/${1:-r06h}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -rf --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; exit 1; }
for v in default RSAMD_TUP_TW=1 RSAMD_TUP_TW=2 default; do
  if [ "$v" = default ]; then e=""; else e="$v"; fi
  echo "== $v"; env $e timeout -k 10 120 python3 tools/probe_np_c2.py --reps 8 --split | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(min(d['wall_ms']), d['split_ms']['tuples'], d['split_ms']['parse_total'])" || exit 1
done
if [ -n "$2" ]; then  # E5 A/B: the product against lib_ab/$2
  for p in 1 2; do
    echo -n "product "; timeout -k 10 120 python3 tools/probe_e5.py || exit 1
    echo -n "$2 "; RSAMD_LIB=$(pwd)/tsbb15-3d-reconstruction-project_amd/lib_ab/$2/librsamd.so timeout -k 10 120 python3 tools/probe_e5.py || exit 1
  done
fi
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail $OUT/bench.err; exit 1; }
echo bench ok
