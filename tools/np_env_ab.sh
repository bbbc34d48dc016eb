#!/bin/bash
# Parity-stream probe (checked against the host replay) under several environment settings,
# interleaved twice.  Usage (through gpurun): bash tools/np_env_ab.sh <tag> "VAR=a" "VAR=b" ...
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for rep in 1 2; do
  for e in "$@"; do
    env $e timeout -k 10 200 python3 tools/np_kw_probe.py > $OUT/probe.tmp 2> $OUT/probe.err || { echo "probe $e failed"; tail -5 $OUT/probe.err; exit 1; }
    sed "s|^|$e rep$rep |" $OUT/probe.tmp | tee -a $OUT/probe.txt
  done
done
