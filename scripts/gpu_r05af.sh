#!/bin/bash
# bf16-operand modality projections (X' / dZ bf16, W_proj copies): GPU parity (bf16 GEMM, C5 bench
# path, bf16 / train-mode suites), then C5 A/B against MMF_NO_PROJ_B16=1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05af}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gemm_bf16.py tests/test_gpu_c5_bench.py tests/test_gpu_bf16.py tests/test_gpu_train_mode.py > $O/pytest.log 2>&1 || exit $?
B="python bench.py --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu"
for i in 1 2; do
  timeout -k 10 200 $B > $O/c5_pb16_$i.json 2> $O/c5_pb16_$i.err || exit $?
  timeout -k 10 200 env MMF_NO_PROJ_B16=1 $B > $O/c5_fp32op_$i.json 2> $O/c5_fp32op_$i.err || exit $?
done
echo done
