#!/bin/bash
# 128 x 256 tiles by default for long-K RK x KR bf16 calls (dZ): parity (bf16 GEMM forms, C5 path,
# bf16 suite), C5 bench, and the previous default (MMF_GEMM_WIDE_DZ unset cannot restore it: A/B
# against r05am2's default runs on another box)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05an}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gemm_bf16.py tests/test_gpu_c5_bench.py tests/test_gpu_bf16.py tests/test_gpu_train_mode.py > $O/pytest.log 2>&1 || exit $?
B="python bench.py --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu"
for i in 1 2 3; do
  timeout -k 10 200 $B > $O/c5_$i.json 2> $O/c5_$i.err || exit $?
done
echo done
