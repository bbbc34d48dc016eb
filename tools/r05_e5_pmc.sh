#!/bin/bash
# E5 at the C2 shape: probe per RSAMD_E5_SLICES value, then PMC of k_e5_roots / count.
# Usage (through gpurun): bash tools/r05_e5_pmc.sh <tag>
set -o pipefail
TAG=${1:-r05e5}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for pass in 1 2; do
  for sl in 0 1 3 4; do
    echo "slices $sl pass $pass $(RSAMD_E5_SLICES=$sl timeout -k 10 100 python3 $R/tools/probe_e5.py)"
  done
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_WAIT_INST_ANY SQ_INSTS_LDS --output-format csv -d $OUT/pmc -o p -- python3 $R/tools/probe_e5.py > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/pmc.log; exit 1; }
python3 - <<PY
import csv, glob
v = {}
for r in csv.DictReader(open(glob.glob("$OUT/pmc/*counter_collection.csv")[0])):
    k = r["Kernel_Name"].split("(")[0]
    v.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k, d in v.items():
    if "roots" in k or "count32q" in k or "gj" in k:
        print(k, {c: round(sum(x) / len(x)) for c, x in d.items()})
PY
