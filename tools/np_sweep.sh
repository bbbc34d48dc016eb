#!/bin/bash
# Chunk-length sweep of the parity stream: probe timing + rocprofv3 trace per RSAMD_NP_KW value.
# Usage (through gpurun): bash tools/np_sweep.sh <tag> <kw> [<kw> ...]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
for kw in "$@"; do
  RSAMD_NP_KW=$kw timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/kw$kw -o np -- python3 tools/probe_np_sampler.py > $OUT/kw$kw.jsonl 2> $OUT/kw$kw.err || { echo "kw $kw failed"; tail -5 $OUT/kw$kw.err; exit 1; }
  echo "kw=$kw"; head -1 $OUT/kw$kw.jsonl
done
