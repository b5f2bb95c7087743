#!/bin/bash
# C5: 16-deep ring for the 8-wave weight-stationary Q / K GEMM (MMF_WSR16_NS=16) A/B, parity with it
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05al}
mkdir -p $O
timeout -k 10 300 env MMF_WSR16_NS=16 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_c5_bench.py tests/test_gpu_gemm_bf16.py > $O/pytest_ns16.log 2>&1 || exit $?
B="python bench.py --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu"
for i in 1 2; do
  timeout -k 10 200 $B > $O/c5_ns12_$i.json 2> $O/c5_ns12_$i.err || exit $?
  timeout -k 10 200 env MMF_WSR16_NS=16 $B > $O/c5_ns16_$i.json 2> $O/c5_ns16_$i.err || exit $?
done
echo done
