#!/bin/bash
# A-stationary bf16 GEMM (gemm_ast_b16_kernel) for the concatenated Q / K projections: bf16 GEMM
# tests, the C5 step parity with MMF_QK_CAT=1, C5 A/B (per-pair weight-stationary vs concatenated).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05ac}
mkdir -p $O
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 300 $PT tests/test_gpu_gemm_bf16.py > $O/pytest_gemm.log 2>&1 || exit $?
timeout -k 10 300 env MMF_QK_CAT=1 $PT tests/test_gpu_c5_bench.py > $O/pytest_c5_cat.log 2>&1 || exit $?
B="python bench.py --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu"
for i in 1 2; do
  timeout -k 10 200 $B > $O/c5_wsr$i.json 2> $O/c5_wsr$i.err || exit $?
  timeout -k 10 200 env MMF_QK_CAT=1 $B > $O/c5_cat$i.json 2> $O/c5_cat$i.err || exit $?
done
echo done
