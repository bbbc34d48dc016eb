#!/bin/bash
# Round 5 parse check: np sampler GPU tests on the product, then the C2 parse probe per library
# (product, lib_ab variants given as arguments), two interleaved passes, and the product's chunk
# timeline.  Usage (through gpurun): bash tools/r05_np.sh <tag> [ab-lib ...]
set -o pipefail
TAG=${1:-r05np}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_np_sampler.py tests/test_gpu_full_parity.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_np.log 2>&1 || { echo np tests failed; tail -30 $OUT/pytest_np.log; exit 1; }
tail -n 2 $OUT/pytest_np.log
for pass in 1 2; do
  for v in prod "$@"; do
    if [ $v = prod ]; then unset RSAMD_LIB; else export RSAMD_LIB=$R/tsbb15-3d-reconstruction-project_amd/lib_ab/$v/librsamd.so; fi
    echo "== $v pass $pass" >> $OUT/probe.txt
    NP_ONLY=2000 timeout -k 10 120 python3 tools/np_kw_probe.py >> $OUT/probe.txt 2>> $OUT/probe.err || { echo "probe $v failed"; tail -5 $OUT/probe.err; exit 1; }
    echo "$v $(tail -n 1 $OUT/probe.txt)"
  done
done
unset RSAMD_LIB
timeout -k 10 150 python3 tools/np_timeline.py 2000 100000 4 > $OUT/tl_prod.json 2>> $OUT/tl.err || { echo timeline failed; exit 1; }
python3 - <<PY
import json
r = json.load(open("$OUT/tl_prod.json"))["last_run"]
for k in ("entry_kernel_us", "track_kernel_us", "multi_phase_us", "multi_phase_draws",
          "single_phase_us", "single_phase_draws", "single_cycles_per_draw", "track_dur_us", "last_chunk"):
    print(k, r.get(k))
PY
