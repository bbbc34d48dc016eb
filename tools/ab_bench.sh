#!/bin/bash
# A/B of plan knobs on the bench: each argument is one env assignment list, e.g.
#   bash tools/ab_bench.sh "RSAMD_TIMING=0" "RSAMD_TIMING=1 RSAMD_OVERLAP=0"
# prints value / ms_per_step / count kernel time per configuration.
set -o pipefail
for cfg in "$@"; do
  env $cfg timeout -k 10 120 python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline \
      --no-parity-mode > /tmp/ab.json || { echo "$cfg FAILED"; exit 1; }
  python3 -c "import json,sys; d=json.load(open('/tmp/ab.json')); print(sys.argv[1].ljust(40), round(d['value']/1e6,1), 'Mhyp/s', round(d['ms_per_step']*1e3,1), 'us/step  count', d['kernels_ms']['k_f8_count'])" "$cfg"
done
