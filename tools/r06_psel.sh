#!/bin/bash
# PnP select with vector count loads against lib_ab/pold: PnP GPU tests, then the C3 probe
# (wall per call, solve / count kernel times) alternating.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/${1:-r06_psel}; mkdir -p $OUT
OLD=$(pwd)/tsbb15-3d-reconstruction-project_amd/lib_ab/pold/librsamd.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_pnp.py tests/test_gpu_tables_dropin.py -x -q -rf --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
for v in new old new old; do
  case $v in new) e="";; old) e="RSAMD_LIB=$OLD";; esac
  echo -n "$v: "; env $e timeout -k 10 120 python3 tools/probe_pnp2.py || exit 1
done
