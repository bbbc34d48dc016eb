#!/bin/bash
# Stall / instruction-cache PMC passes over pure solve and pure tail launches.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-pmct}
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
for probe in solve tail; do
  PROBE=$probe timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_IFETCH --output-format csv -d $OUT/sq_$probe -o pmc -- python3 tools/probe_tail_solve.py > $OUT/sq_$probe.log 2>&1 || { echo "sq $probe failed"; exit 1; }
  PROBE=$probe timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_TC_INST_REQ SQC_DCACHE_MISSES --output-format csv -d $OUT/sqc_$probe -o pmc -- python3 tools/probe_tail_solve.py > $OUT/sqc_$probe.log 2>&1 || { echo "sqc $probe failed"; exit 1; }
  PROBE=$probe timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$probe -o kt -- python3 tools/probe_tail_solve.py > $OUT/kt_$probe.log 2>&1 || { echo "kt $probe failed"; exit 1; }
done
ls $OUT
