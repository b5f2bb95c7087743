# fp32 MFMA shape micro-benchmark (32x32x2 vs 16x16x4 at the GEMM's fragment pattern)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-shape}
mkdir -p $O
timeout -k 10 120 scripts/micro/shape_micro > $O/shape_micro.txt 2>&1 || exit 1
cat $O/shape_micro.txt
