#!/bin/bash
# k_np_tuples_wave time per A/B library (lib_ab/<name>), C2 stream, rocprofv3 kernel stats.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-tup}; shift
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for v in "$@"; do
  if [ "$v" = base ]; then L=$R/tsbb15-3d-reconstruction-project_amd/lib/librsamd.so; else L=$R/tsbb15-3d-reconstruction-project_amd/lib_ab/$v/librsamd.so; fi
  RSAMD_LIB=$L NP_ONLY=2000 timeout -k 5 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v -o np -- python3 $R/tools/np_kw_probe.py > $OUT/$v.log 2>&1 || { echo "$v failed"; tail -3 $OUT/$v.log; exit 1; }
  echo "$v $(tail -1 $OUT/$v.log | cut -c1-120)"
  python3 $R/tools/kstats.py $OUT/$v/np_kernel_stats.csv | grep -E "tuples|track|entry|jump|filter"
done
