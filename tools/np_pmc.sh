#!/bin/bash
# PMC passes over the parity-stream kernels (tools/probe_split.py, world 1): one rocprofv3 run
# per counter group.  Usage (gpurun): bash tools/np_pmc.sh <tag> [c2|c5]
set -o pipefail
TAG=$1; CASE=${2:-c2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$CASE" = c5 ]; then ARGS="--n 10000 --outliers 0.6 --seed 5 --hyps 1000000 --worlds 1 --reps 0"; else ARGS="--worlds 1 --reps 1"; fi
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_SCA"
G2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INST_CYCLES_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"
i=0
G3="FETCH_SIZE"
G4="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
for g in "$G1" "$G2" "$G3" "$G4"; do
  i=$((i+1))
  ( cd /tmp && timeout -s KILL 200 rocprofv3 --pmc $g --output-format csv -d $OUT/pmc$i -o pmc -- python3 $R/tools/probe_split.py $ARGS > $OUT/pmc$i.log 2>&1 ) || { echo "pass $i failed"; tail -5 $OUT/pmc$i.log; exit 1; }
done
python3 $R/tools/pmc_kernels.py $OUT/pmc1 $OUT/pmc2 $OUT/pmc3 $OUT/pmc4 > $OUT/pmc_summary.txt 2>&1 || true
cat $OUT/pmc_summary.txt
