#!/bin/bash
# Entry kernel compacted in place (4 n1p bytes of LDS) against lib_ab/eold (8 n1p): stream
# parity tests, the C5 chunk timeline, C2 / C5 parity-run A/B.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/${1:-r06_entry}; mkdir -p $OUT
OLD=$(pwd)/tsbb15-3d-reconstruction-project_amd/lib_ab/eold/librsamd.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_np_sampler.py tests/test_gpu_np_shard.py tests/test_gpu_full_parity.py -x -q -rf --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python3 tools/np_timeline.py 10000 1000000 1 > $OUT/c5_timeline.json || exit 1
python3 -c "import json; d=json.load(open('$OUT/c5_timeline.json'))['last_run']; print('c5 entry', d['entry_kernel_us'], d['entry_start_skew_us'], 'track', d['track_kernel_us'])"
for cfg in "" "--n 10000 --hyps 1000000 --outliers 0.6 --seed 5"; do
  for v in new old new old; do
    case $v in new) e="";; old) e="RSAMD_LIB=$OLD";; esac
    echo -n "[$cfg] $v: "; env $e timeout -k 10 120 python3 tools/probe_np_c2.py --reps 6 --split $cfg | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); w=sorted(d['wall_ms'][2:]); print(round(w[0],3), round(w[len(w)//2],3), d['best_index'], d['best_count'], 'entry', round(d['split_ms']['entry'],3), 'track', round(d['split_ms']['track'],3))" || exit 1
  done
done
