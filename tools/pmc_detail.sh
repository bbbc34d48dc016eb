#!/bin/bash
# Detailed SQ counters of the counting kernels (fp32 / fp64) on the C2 workload.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_detail
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
for mode in ${MODES:-x fp32}; do
  for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
             "SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE GRBM_COUNT" \
             "SQ_INSTS_SMEM SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_REQ SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH"; do
    tag=$(echo $set | cut -c1-12 | tr ' ' '_')
    RSAMD_COUNT=$mode timeout -k 10 200 rocprofv3 --pmc $set --output-format csv -d $OUT/${mode}_$tag -o p -- python3 tools/sweep.py > $OUT/${mode}_$tag.log 2>&1 || echo "pass $mode $tag failed"
  done
done
python3 - <<'PY'
import csv, glob, os, collections
out = os.environ.get("GRAFT_REPO_ROOT", ".") + "/gpurun_out/pmc_detail"
for f in sorted(glob.glob(out + "/*/p_counter_collection.csv")):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "count" in r["Kernel_Name"] and "max" not in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(os.path.basename(os.path.dirname(f)), {k: round(sum(v) / len(v)) for k, v in agg.items()})
PY
