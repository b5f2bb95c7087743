#!/bin/bash
# C5: 4-deep LDS ring for the bf16 RK-A GEMM forms (projection, dZ, dX) A/B (MMF_GEMM_B16_NS4=1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05ai}
mkdir -p $O
timeout -k 10 300 env MMF_GEMM_B16_NS4=1 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_c5_bench.py > $O/pytest_ns4.log 2>&1 || exit $?
B="python bench.py --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu"
for i in 1 2; do
  timeout -k 10 200 $B > $O/c5_ns3_$i.json 2> $O/c5_ns3_$i.err || exit $?
  timeout -k 10 200 env MMF_GEMM_B16_NS4=1 $B > $O/c5_ns4_$i.json 2> $O/c5_ns4_$i.err || exit $?
done
echo done
