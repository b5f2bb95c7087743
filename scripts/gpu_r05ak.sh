#!/bin/bash
# dZ GEMM gate from the bf16 P copy (EPI_GATE_B16): C5 parity + bf16 suites, C5 A/B against MMF_NO_GATE_B16=1
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05ak}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_c5_bench.py tests/test_gpu_bf16.py tests/test_gpu_gemm_bf16.py > $O/pytest.log 2>&1 || exit $?
B="python bench.py --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu"
for i in 1 2; do
  timeout -k 10 200 $B > $O/c5_gb16_$i.json 2> $O/c5_gb16_$i.err || exit $?
  timeout -k 10 200 env MMF_NO_GATE_B16=1 $B > $O/c5_g32_$i.json 2> $O/c5_g32_$i.err || exit $?
done
echo done
