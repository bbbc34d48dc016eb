#!/bin/bash
# One GPU-box session: tests, smoke, bench, rocprofv3 kernel trace + PMC passes.
# Usage (through gpurun): bash tools/gpu_round.sh <tag> [steps]
set -o pipefail
TAG=${1:-r01}
STEPS=${2:-100}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
echo "pytest_gpu exit $?" | tee -a $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; exit 1; }
timeout -k 10 400 python bench.py --steps $STEPS --warmup 200 > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; exit 1; }
cat $OUT/bench.json
# kernel trace of the C2 headline alone (no parity mode, fp64 count or extras: every
# k_f8_count32q launch in it is a C2-size launch, so the stats average is the line's kernel)
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --steps $STEPS --warmup 200 --no-cpu-baseline --no-extras --no-parity-mode --no-fp64-count > $OUT/prof_bench.log 2>&1 || { echo rocprof failed; exit 1; }
# and the whole line's kernels (parity mode and its split projection included) for reference
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_all -o bench -- python3 bench.py --steps $STEPS --warmup 200 --no-cpu-baseline --no-extras > $OUT/prof_all.log 2>&1 || { echo rocprof all failed; exit 1; }
# PMC passes on a warmed, clock-ramped run (200 warm-up launches, 50 counted), one pass per
# counter block (MI355X_MICROARCH.md: FETCH_SIZE alone, WRITE_SIZE alone)
B="python3 bench.py --steps 50 --warmup 200 --no-cpu-baseline --no-parity-mode --no-extras --no-fp64-count"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o pmc -- $B > $OUT/pmc_fetch.log 2>&1 || { echo pmc fetch failed; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_write -o pmc -- $B > $OUT/pmc_write.log 2>&1 || { echo pmc write failed; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_FMA_F64 --output-format csv -d $OUT/pmc_sq -o pmc -- $B > $OUT/pmc_sq.log 2>&1 || echo "pmc sq failed"
# scalar / instruction cache pass: the count kernel reads its points through the scalar cache
timeout -s KILL 300 rocprofv3 --pmc SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_ICACHE_REQ SQC_ICACHE_MISSES SQC_TC_DATA_READ_REQ SQC_TC_INST_REQ GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_sqc -o pmc -- $B > $OUT/pmc_sqc.log 2>&1 || echo "pmc sqc failed"
find $OUT -name "*.csv" | head -50
