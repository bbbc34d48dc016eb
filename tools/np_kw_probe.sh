#!/bin/bash
# tools/np_kw_probe.py per chunk length ("-" = automatic).  Usage: bash tools/np_kw_probe.sh <tag> kw...
TAG=${1:-kw}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for kw in "$@"; do
  if [ "$kw" = "-" ]; then unset RSAMD_NP_KW; else export RSAMD_NP_KW=$kw; fi
  timeout -k 10 150 python3 tools/np_kw_probe.py >> $OUT/probe.jsonl 2>> $OUT/probe.err || { echo "kw $kw failed"; tail -5 $OUT/probe.err; exit 1; }
done
cat $OUT/probe.jsonl
