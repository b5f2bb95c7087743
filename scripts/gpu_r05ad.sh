#!/bin/bash
# A-stationary GEMM with an 8-deep B ring (libmmfusion_ast8.so) in the concatenated Q / K mode
# against the per-pair weight-stationary product.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05ad}
mkdir -p $O
L=multimodal-sensor-fusion-with-attention-rajeevatla_amd/csrc/libmmfusion_ast8.so
timeout -k 10 300 env MMF_LIB_PATH=$L python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gemm_bf16.py > $O/pytest_gemm.log 2>&1 || exit $?
B="python bench.py --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu"
for i in 1 2; do
  timeout -k 10 200 $B > $O/c5_wsr$i.json 2> $O/c5_wsr$i.err || exit $?
  timeout -k 10 200 env MMF_QK_CAT=1 MMF_LIB_PATH=$L $B > $O/c5_cat8_$i.json 2> $O/c5_cat8_$i.err || exit $?
done
echo done
