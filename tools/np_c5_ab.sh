#!/bin/bash
# C5 parity-mode A/B over parse layout knobs: each argument is an env assignment list (or
# "default"), run as a separate probe process (tools/probe_np_c2.py, C5, step split).
# Usage (gpurun): bash tools/np_c5_ab.sh "default" "RSAMD_NP_CPR=512" ...
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
for v in "$@"; do
  if [ "$v" = default ]; then e=""; else e="$v"; fi
  echo "== $v"
  env $e timeout -k 10 200 python3 tools/probe_np_c2.py --n 10000 --hyps 1000000 --outliers 0.6 --seed 5 --reps 2 --split || exit 1
done
