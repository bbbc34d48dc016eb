#!/bin/bash
# Counting-kernel pool A/B: correctness on the product setting, then the headline bench per
# RSAMD_QPOOL[:RSAMD_QCHUNK] setting, interleaved twice; timeline of the first setting.
set -o pipefail
TAG=${1:-cpool}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_full_parity.py tests/test_gpu_f8.py -q -x --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
st=$?; tail -2 $OUT/pytest.log; [ $st -eq 0 ] || exit 1
for rep in 1 2; do
for cfg in "$@"; do
  pool=${cfg%%:*}; chunk=64; [ "$cfg" != "$pool" ] && chunk=${cfg#*:}
  RSAMD_QPOOL=$pool RSAMD_QCHUNK=$chunk timeout -k 10 200 python bench.py --steps 200 --warmup 200 --no-extras --no-parity-mode --no-cpu-baseline --no-fp64-count > $OUT/b.json 2> $OUT/b.err || { echo "$cfg failed"; tail -3 $OUT/b.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b.json'));print('pool $cfg rep$rep', round(d['value']/1e6,1), round(d['roofline']['per_launch']['avg_ms']*1e3,2), round(d['roofline']['frac'],4))" | tee -a $OUT/ab.txt
done
done
cfg=$1; pool=${cfg%%:*}; chunk=64; [ "$cfg" != "$pool" ] && chunk=${cfg#*:}
RSAMD_QPOOL=$pool RSAMD_QCHUNK=$chunk RSAMD_TSTAMP=/tmp/ts.bin timeout -k 10 200 python tools/count_timeline.py > $OUT/timeline.txt 2>&1 || echo "timeline failed"
head -2 $OUT/timeline.txt
