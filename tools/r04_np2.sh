#!/bin/bash
# Parse A/B: product (multi-trajectory windows via fast_window), lib_ab/one_valu (single too),
# lib_ab/base (round-3 windows): np sampler tests on the product, then C2 / N=10k probe and the
# C2 chunk timeline per variant.  Usage (through gpurun): bash tools/r04_np2.sh <tag>
set -o pipefail
TAG=${1:-r04np2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
RSAMD_LIB=$R/tsbb15-3d-reconstruction-project_amd/lib_ab/w14ls/librsamd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_full_parity.py tests/test_gpu_np_shard.py -k "c2 or projection" -x -q --timeout 200 --timeout-method thread > $OUT/pytest_np.log 2>&1 || { echo np tests failed; tail -30 $OUT/pytest_np.log; exit 1; }
tail -2 $OUT/pytest_np.log
for pass in 1 2; do
for v in prod w14ls w12ls; do
  if [ $v = prod ]; then unset RSAMD_LIB; else export RSAMD_LIB=$R/tsbb15-3d-reconstruction-project_amd/lib_ab/$v/librsamd.so; fi
  echo "== $v pass $pass" | tee -a $OUT/probe.txt
  NP_ONLY=2000 timeout -k 10 150 python tools/np_kw_probe.py >> $OUT/probe.txt 2>&1 || { echo probe failed; tail $OUT/probe.txt; exit 1; }
  if [ $pass = 1 ]; then timeout -k 10 150 python tools/np_timeline.py 2000 100000 4 > $OUT/tl_$v.json 2>> $OUT/tl.err || { echo timeline failed; exit 1; }; fi
done
done
unset RSAMD_LIB
cat $OUT/probe.txt
python - <<PY
import json
for v in ("prod", "w14ls", "w12ls"):
    r = json.load(open("$OUT/tl_%s.json" % v))["last_run"]
    print(v, "entry", r["entry_kernel_us"], "track", r["track_kernel_us"], "multi", r["multi_phase_us"], "single", r["single_phase_us"], "cpd", r["single_cycles_per_draw"])
PY
