#!/bin/bash
# PnP stop-tolerance A/B: accuracy against numpy's SVD and the PnP tests with lib_ab/tol13, then
# the C3 timing A/B.  Usage (gpurun): bash tools/pnp_tol_ab.sh
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
L=$(pwd)/tsbb15-3d-reconstruction-project_amd/lib_ab/${1:-tol13}/librsamd.so
K="tests/test_gpu_pnp.py::test_dlt_minimal_samples_accuracy_against_numpy_svd"
timeout -k 10 200 python -u -m pytest -s -q $K --timeout 150 --timeout-method thread 2>&1 | grep -E "DLT vs|passed|failed" || exit 1
RSAMD_LIB=$L timeout -k 10 300 python -u -m pytest -s -q tests/test_gpu_pnp.py tests/test_gpu_tables_dropin.py -x --timeout 200 --timeout-method thread 2>&1 | grep -E "DLT vs|passed|failed" || exit 1
bash tools/pnp_ab.sh ${1:-tol13} | grep -o '"lib[^R]*'
