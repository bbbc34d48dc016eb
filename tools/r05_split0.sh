set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05split0; mkdir -p $OUT; export TMPDIR=/tmp; cd /tmp
RSAMD_NP_SPLIT=0 NP_ONLY=2000 timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o np -- python3 $R/tools/np_kw_probe.py > $OUT/prof.log 2>&1 || { echo fail; tail -5 $OUT/prof.log; exit 1; }
grep gpu_ms $OUT/prof.log
python3 $R/tools/r05_np_timeline.py $OUT/prof/np_kernel_trace.csv
