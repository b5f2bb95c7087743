# Phase stamps of the pooled attention kernels (diagnostic builds) + the GEMM micro-benchmark.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-stamps}
mkdir -p $O
C=multimodal-sensor-fusion-with-attention-rajeevatla_amd/csrc
MMF_LIB_PATH=$C/libmmfusion_stamps.so timeout -k 10 200 python -u scripts/attn_stamps.py attn > $O/stamps_bwd.json 2> $O/stamps_bwd.err || exit 1
MMF_LIB_PATH=$C/libmmfusion_stampsf.so timeout -k 10 200 python -u scripts/attn_stamps.py fwd > $O/stamps_fwd.json 2> $O/stamps_fwd.err || exit 1
timeout -k 10 120 scripts/micro/gemm_micro > $O/gemm_micro.txt 2>&1 || exit 1
echo done
