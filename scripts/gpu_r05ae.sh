#!/bin/bash
# 8-wave weight-stationary bf16 projection GEMM over 256-column groups (libmmfusion_w8.so): bf16
# GEMM + C5 parity with it, C5 A/B against the 4-wave / 128-column product.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05ae}
mkdir -p $O
L=multimodal-sensor-fusion-with-attention-rajeevatla_amd/csrc/libmmfusion_w8.so
timeout -k 10 400 env MMF_LIB_PATH=$L python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gemm_bf16.py tests/test_gpu_c5_bench.py > $O/pytest_w8.log 2>&1 || exit $?
B="python bench.py --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu"
for i in 1 2; do
  timeout -k 10 200 $B > $O/c5_w4_$i.json 2> $O/c5_w4_$i.err || exit $?
  timeout -k 10 200 env MMF_LIB_PATH=$L $B > $O/c5_w8_$i.json 2> $O/c5_w8_$i.err || exit $?
done
echo done
