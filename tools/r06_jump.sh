#!/bin/bash
# The ring form of the jump (k_mt_jump_slide) against the prefix form (RSAMD_JUMP_PREFIX=1):
# stream parity tests, C2 / C5 parity-run A/B, and a kernel trace of C2 probes of each.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/${1:-r06_jump}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_np_sampler.py tests/test_gpu_np_shard.py tests/test_gpu_full_parity.py -x -q -rf --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
for cfg in "" "--n 10000 --hyps 1000000 --outliers 0.6 --seed 5"; do
  for v in default RSAMD_JUMP_PREFIX=1 default RSAMD_JUMP_PREFIX=1; do
    if [ "$v" = default ]; then e=""; else e="$v"; fi
    echo -n "[$cfg] $v: "; env $e timeout -k 10 120 python3 tools/probe_np_c2.py --reps 8 --split $cfg | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); w=sorted(d['wall_ms'][2:]); print(round(w[0],3), round(w[len(w)//2],3), d['best_index'], d['best_count'], 'jump', round(d['split_ms']['jump'],3))" || exit 1
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr_slide -o t -- python3 tools/probe_np_c2.py --reps 3 > $OUT/tr_slide.log 2>&1 || exit 1
RSAMD_JUMP_PREFIX=1 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr_prefix -o t -- python3 tools/probe_np_c2.py --reps 3 > $OUT/tr_prefix.log 2>&1 || exit 1
for d in tr_slide tr_prefix; do
  echo "== $d"; python3 - $(find $OUT/$d -name "*kernel_trace.csv") <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if 'k_mt_jump' in r['Kernel_Name']]
for r in rows[-3:]:
    print(r['Grid_Size_X'] if 'Grid_Size_X' in r else r.get('Grid_Size'), (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3, 'us')
PY
done
