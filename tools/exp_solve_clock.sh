#!/bin/bash
# Solve-time breakdown (RSAMD_SOLVE_DIAG variants), effective clock of the counting kernel
# (GRBM_GUI_ACTIVE pass) and a 2-rank bench rehearsal on one GPU (gloo record exchange).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-exp}
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
for d in 0 1 2 3 4 7; do
  echo -n "diag=$d " >> $OUT/solve_split.txt
  RSAMD_SOLVE_DIAG=$d timeout -k 10 120 python3 tools/solve_split.py >> $OUT/solve_split.txt 2>&1 || { echo "solve_split $d failed"; exit 1; }
done
cat $OUT/solve_split.txt
timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU SQ_WAVES --output-format csv -d $OUT/pmc_clock -o pmc -- python3 tools/clock_probe.py > $OUT/pmc_clock.log 2>&1 || { echo "clock pmc failed"; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_clock -o clk -- python3 tools/clock_probe.py > $OUT/prof_clock.log 2>&1 || { echo "clock trace failed"; exit 1; }
RSAMD_BENCH_DEVICE=0 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > $OUT/bench2.json 2> $OUT/bench2.err || { echo "2-rank bench failed"; tail -30 $OUT/bench2.err; exit 1; }
cat $OUT/bench2.json
