#!/bin/bash
# PMC passes of the counting kernel on a warmed bench (200 warm-up runs, 50 timed), one pass per
# counter group; RSAMD_COUNT selects the variant (default: the product kernel).
set -o pipefail
TAG=${1:-cpm}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
B="python3 bench.py --steps 50 --warmup 200 --no-extras --no-parity-mode --no-cpu-baseline --no-fp64-count"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/pmc_sq -o pmc -- $B > $OUT/pmc_sq.log 2>&1 || { echo sq failed; tail $OUT/pmc_sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_INST_CYCLES_SALU --output-format csv -d $OUT/pmc_sq2 -o pmc -- $B > $OUT/pmc_sq2.log 2>&1 || { echo sq2 failed; tail $OUT/pmc_sq2.log; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o pmc -- $B > $OUT/pmc_fetch.log 2>&1 || { echo fetch failed; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_write -o pmc -- $B > $OUT/pmc_write.log 2>&1 || { echo write failed; exit 1; }
echo ok
