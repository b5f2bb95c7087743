#!/bin/bash
# weight-stationary bf16 Q/K projections (C5 "medium"): the bf16 GEMM forms alone, the medium-precision parity
# tests, then the C5 line A/B (gemm_wsr_b16_kernel vs MMF_NO_WSR16=1) with rocprofv3 stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05j}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_bf16.py -v --timeout 120 --timeout-method thread > $O/pytest_gemm.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gemm.log
if [ $rc -ne 0 ]; then echo "bf16 GEMM tests failed rc=$rc: stopping"; exit 1; fi
timeout -k 10 600 python -u -m pytest tests/test_gpu_c5_bench.py tests/test_gpu_bf16.py tests/test_gpu_train_mode.py -v --timeout 300 --timeout-method thread > $O/pytest_medium.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_medium.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed rc=$rc"; exit $rc; fi
grep -q "illegal memory access\|Memory access fault" $O/pytest_medium.log && { echo "GPU fault: stopping"; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu > $O/c5_a$i.json 2> $O/c5_a$i.err || exit $?
  MMF_NO_WSR16=1 timeout -k 10 300 python bench.py --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu > $O/c5_b$i.json 2> $O/c5_b$i.err || exit $?
done
bash scripts/gpu_prof.sh $O c5_medium --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu || exit $?
echo done
