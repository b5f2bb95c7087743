set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-gm}
mkdir -p $O
timeout -k 10 120 scripts/micro/gemm_micro > $O/gemm_micro.txt 2>&1 || exit 1
cat $O/gemm_micro.txt
