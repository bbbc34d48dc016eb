#!/bin/bash
# GPU tests + smoke, then the C2 / C5 parity-run A/B: the F run queued behind the parse
# (default) against the parse waited for first (RSAMD_NP_SYNC=1).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/${1:-r06_async}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -rf --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; exit 1; }
for cfg in "" "--n 10000 --hyps 1000000 --outliers 0.6 --seed 5"; do
  for v in default RSAMD_NP_SYNC=1 default RSAMD_NP_SYNC=1; do
    if [ "$v" = default ]; then e=""; else e="$v"; fi
    echo -n "[$cfg] $v: "; env $e timeout -k 10 120 python3 tools/probe_np_c2.py --reps 12 $cfg | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); w=sorted(d['wall_ms'][2:]); print(round(w[0],3), round(w[len(w)//2],3), d['best_index'], d['best_count'])" || exit 1
  done
done
