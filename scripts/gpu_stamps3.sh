set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-stamps3}
mkdir -p $O
C=multimodal-sensor-fusion-with-attention-rajeevatla_amd/csrc
STAMPS_WARM=2000 MMF_LIB_PATH=$C/libmmfusion_stamps.so timeout -k 10 200 python -u scripts/attn_stamps.py attn > $O/stamps_bwd_warm.json 2> $O/e1.err || exit 1
STAMPS_WARM=2000 MMF_LIB_PATH=$C/libmmfusion_stampsf.so timeout -k 10 200 python -u scripts/attn_stamps.py fwd > $O/stamps_fwd_warm.json 2> $O/e3.err || exit 1
echo done
