#!/bin/bash
# XCD-aware slice order vs the previous order (lib_ab/base0): correctness, interleaved bench,
# and HBM FETCH/WRITE per counting launch for both (one PMC pass per counter).
set -o pipefail
TAG=${1:-cxcd}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_full_parity.py tests/test_gpu_f8.py -q -x --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
st=$?; tail -2 $OUT/pytest.log; [ $st -eq 0 ] || exit 1
bash tools/count_lib_ab.sh $TAG base0=base0 xcd=base || exit 1
B="python3 bench.py --steps 50 --warmup 200 --no-cpu-baseline --no-parity-mode --no-extras --no-fp64-count"
for v in base0 xcd; do
  L=$R/tsbb15-3d-reconstruction-project_amd/lib/librsamd.so
  [ $v = base0 ] && L=$R/tsbb15-3d-reconstruction-project_amd/lib_ab/base0/librsamd.so
  RSAMD_LIB=$L timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/f_$v -o pmc -- $B > $OUT/f_$v.log 2>&1 || { echo "fetch $v failed"; exit 1; }
  RSAMD_LIB=$L timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/w_$v -o pmc -- $B > $OUT/w_$v.log 2>&1 || { echo "write $v failed"; exit 1; }
  echo "== $v"; python3 tools/pmc_read.py $OUT/f_$v k_f8_count32q; python3 tools/pmc_read.py $OUT/w_$v k_f8_count32q
done
