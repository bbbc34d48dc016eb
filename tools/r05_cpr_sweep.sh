#!/bin/bash
# Round 5: C2 parse time against the chunk count (RSAMD_NP_CPR) and the tracking workgroup's
# waves (lib_ab/w<k>, RSAMD_TRACK_WAVES=k), two interleaved passes; then the product's chunk
# timeline.  Usage (through gpurun): bash tools/r05_cpr_sweep.sh <tag>
set -o pipefail
TAG=${1:-r05cpr}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
AB=$R/tsbb15-3d-reconstruction-project_amd/lib_ab
run() {  # <label> <lib or -> <cpr or ->
  if [ "$2" = "-" ]; then unset RSAMD_LIB; else export RSAMD_LIB=$AB/$2/librsamd.so; fi
  if [ "$3" = "-" ]; then unset RSAMD_NP_CPR; else export RSAMD_NP_CPR=$3; fi
  echo "== $1 lib=$2 cpr=$3" >> $OUT/probe.txt
  NP_ONLY=2000 timeout -k 10 120 python3 tools/np_kw_probe.py >> $OUT/probe.txt 2>> $OUT/probe.err || { echo "probe $1 failed"; tail -5 $OUT/probe.err; exit 1; }
  tail -n 1 $OUT/probe.txt
}
for pass in 1 2; do
  run prod - - || exit 1
  run prod384 - 384 || exit 1
  run prod640 - 640 || exit 1
  run prod768 - 768 || exit 1
  run w12_512 w12 512 || exit 1
  run w10_768 w10 768 || exit 1
  run w8_1024 w8 1024 || exit 1
  run w8_768 w8 768 || exit 1
done
unset RSAMD_LIB RSAMD_NP_CPR
timeout -k 10 150 python3 tools/np_timeline.py 2000 100000 4 > $OUT/tl_prod.json 2>> $OUT/tl.err || { echo timeline failed; exit 1; }
python3 - <<PY
import json
r = json.load(open("$OUT/tl_prod.json"))["last_run"]
for k in ("entry_kernel_us", "track_kernel_us", "entry_dur_us", "multi_phase_us", "multi_phase_draws",
          "single_phase_us", "single_phase_draws", "single_cycles_per_draw", "track_dur_us", "last_chunk"):
    print(k, r.get(k))
PY
