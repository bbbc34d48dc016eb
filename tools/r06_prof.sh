#!/bin/bash
# Round-6 profile session: gpu_round.sh (tests, smoke, bench, C2-only and whole-line kernel
# traces, PMC passes of the counting kernel) then the calibrated traffic (r06_traffic.sh).
# Usage (gpurun): bash tools/r06_prof.sh <tag>
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_round.sh $TAG 100 > gpurun_out/${TAG}_round.log 2>&1 || { echo "gpu_round failed"; tail -20 gpurun_out/${TAG}_round.log; exit 1; }
echo round ok; grep "pytest_gpu exit" gpurun_out/$TAG/pytest_gpu.log
bash tools/r06_traffic.sh $TAG/traffic > gpurun_out/${TAG}_traffic.log 2>&1 || { echo "traffic failed"; tail -20 gpurun_out/${TAG}_traffic.log; exit 1; }
echo traffic ok
