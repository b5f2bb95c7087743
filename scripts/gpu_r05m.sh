#!/bin/bash
# gemm_wsr_b16_kernel ring depth A/B on C5 "medium": 9 tiles (product) vs 6 (MMF_WSR16_NS=6).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05m}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_bf16.py tests/test_gpu_c5_bench.py -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log
if [ $rc -ne 0 ]; then echo "tests failed rc=$rc: stopping"; exit 1; fi
for i in 1 2; do
  timeout -k 10 300 python bench.py --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu > $O/c5_a$i.json 2> $O/c5_a$i.err || exit $?
  MMF_WSR16_NS=6 timeout -k 10 300 python bench.py --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu > $O/c5_b$i.json 2> $O/c5_b$i.err || exit $?
done
echo done
