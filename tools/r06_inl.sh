#!/bin/bash
# GPU tests, then C2 / C3-size parity-run A/B: S_RANSAC written to pinned host memory by the
# tail (product) against lib_ab/hold (copied after the run).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/${1:-r06_inl}; mkdir -p $OUT
OLD=$(pwd)/tsbb15-3d-reconstruction-project_amd/lib_ab/hold/librsamd.so
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -rf --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
for v in new old new old; do
  case $v in new) e="";; old) e="RSAMD_LIB=$OLD";; esac
  echo -n "$v: "; env $e timeout -k 10 120 python3 tools/probe_np_c2.py --reps 12 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); w=sorted(d['wall_ms'][2:]); print(round(w[0],3), round(w[len(w)//2],3), d['best_index'], d['best_count'])" || exit 1
done
