#!/bin/bash
# Count kernel A/B (product vs lib_ab/<variant>): C2 bench lines (headline only), a C2-only
# kernel trace and the WRITE_SIZE / FETCH_SIZE passes per library, interleaved twice.
# Usage (through gpurun): bash tools/r05_count_ab.sh <tag> <variant...>
set -o pipefail
TAG=${1:-r05cab}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
B="python3 $R/bench.py --steps 200 --warmup 300 --no-cpu-baseline --no-parity-mode --no-extras --no-fp64-count"
for pass in 1 2; do
  for v in prod "$@"; do
    if [ $v = prod ]; then unset RSAMD_LIB; else export RSAMD_LIB=$R/tsbb15-3d-reconstruction-project_amd/lib_ab/$v/librsamd.so; fi
    timeout -k 10 200 $B > $OUT/bench_${v}_$pass.json 2>> $OUT/bench.err || { echo "bench $v failed"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/bench_${v}_$pass.json')); print('$v pass $pass', round(d['value']/1e6,1), 'Mhyp/s count_ms', round(d['kernels_ms']['k_f8_count32q'],5))"
  done
done
cd /tmp
for v in prod "$@"; do
  if [ $v = prod ]; then unset RSAMD_LIB; else export RSAMD_LIB=$R/tsbb15-3d-reconstruction-project_amd/lib_ab/$v/librsamd.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$v -o k -- $B > $OUT/prof_$v.log 2>&1 || { echo "rocprof $v failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmcw_$v -o p -- $B > $OUT/pmcw_$v.log 2>&1 || { echo "pmc w $v failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmcf_$v -o p -- $B > $OUT/pmcf_$v.log 2>&1 || { echo "pmc f $v failed"; exit 1; }
  python3 - <<PY
import csv, glob
def per(path, name):
    v = {}
    for r in csv.DictReader(open(glob.glob(path)[0])):
        if "k_f8_count32q" in r["Kernel_Name"]:
            v.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: sum(x) / len(x) for k, x in v.items()}
tr = [r for r in csv.DictReader(open(glob.glob("$OUT/prof_$v/*kernel_trace.csv")[0])) if "k_f8_count32q" in r["Kernel_Name"]]
d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tr]
w = per("$OUT/pmcw_$v/*counter_collection.csv", "w"); f = per("$OUT/pmcf_$v/*counter_collection.csv", "f")
print("$v", "rocprof avg us %.2f (timed %.2f) over %d" % (sum(d) / len(d) / 1e3, sum(d[-200:]) / 200 / 1e3, len(d)),
      "WRITE MB %.3f FETCH MB %.3f" % (w.get("WRITE_SIZE", 0) * 1024 / 1e6, f.get("FETCH_SIZE", 0) * 1024 / 1e6))
PY
done
