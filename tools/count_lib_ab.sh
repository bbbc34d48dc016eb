#!/bin/bash
# Counting-kernel A/B over libraries and env settings, interleaved twice: headline bench
# (HIP-event kernel time).  Args: name=libdir[:ENV=VAL,...]  ("base" = the product library)
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-clab}; shift
mkdir -p $OUT
cd $R
for rep in 1 2; do
for spec in "$@"; do
  name=${spec%%=*}; rest=${spec#*=}; lib=${rest%%:*}; envs=""
  [ "$rest" != "$lib" ] && envs=$(echo ${rest#*:} | tr ',' ' ')
  if [ "$lib" = base ]; then L=$R/tsbb15-3d-reconstruction-project_amd/lib/librsamd.so; else L=$R/tsbb15-3d-reconstruction-project_amd/lib_ab/$lib/librsamd.so; fi
  env RSAMD_LIB=$L $envs timeout -k 10 200 python bench.py --steps 200 --warmup 200 --no-extras --no-parity-mode --no-cpu-baseline --no-fp64-count > $OUT/b_$name.json 2> $OUT/b_$name.err || { echo "$name failed"; tail -3 $OUT/b_$name.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b_$name.json'));print('$name', round(d['value']/1e6,1), round(d['roofline']['per_launch']['avg_ms']*1e3,2), round(d['roofline']['frac'],4))"
done
done
