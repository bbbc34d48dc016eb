#!/bin/bash
# Parity parse time (tools/probe_np_scaling.py) per parse chunk length (RSAMD_NP_KW; "-" is the
# automatic choice), after the sampler tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_np_sampler.py tests/test_gpu_full_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/npkw_pytest.log 2>&1
st=$?; tail -2 gpurun_out/npkw_pytest.log; [ $st -eq 0 ] || exit 1
for kw in "$@"; do
  if [ "$kw" = "-" ]; then e=""; else e="RSAMD_NP_KW=$kw"; fi
  echo "kw $kw"
  env $e timeout -k 10 120 python tools/probe_np_scaling.py || exit 1
done
