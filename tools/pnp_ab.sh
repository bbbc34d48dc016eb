#!/bin/bash
# PnP solve A/B: the product library against lib_ab/<name> variants (tools/probe_pnp2.py).
# Usage (gpurun): bash tools/pnp_ab.sh [test] name...
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
if [ "$1" = "test" ]; then
  shift
  timeout -k 10 300 python -u -m pytest tests/test_gpu_pnp.py tests/test_gpu_tables_dropin.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pnp_ab_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/pnp_ab_pytest.log; [ $rc -eq 0 ] || exit 1
fi
for i in 1 2; do
  timeout -k 10 120 python3 tools/probe_pnp2.py || exit 1
  for n in "$@"; do
    RSAMD_LIB=$(pwd)/tsbb15-3d-reconstruction-project_amd/lib_ab/$n/librsamd.so timeout -k 10 120 python3 tools/probe_pnp2.py || exit 1
  done
done
