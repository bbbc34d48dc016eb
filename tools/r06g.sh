set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/r06_np.sh r06g || exit 1
bash tools/np_c5_ab.sh default "RSAMD_NP_CPR=512" "RSAMD_NP_CPR=768" > gpurun_out/r06g/c5ab.txt 2>&1 || { tail -5 gpurun_out/r06g/c5ab.txt; exit 1; }
cat gpurun_out/r06g/c5ab.txt
