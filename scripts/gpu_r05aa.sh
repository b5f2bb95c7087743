#!/bin/bash
# 128 x 256 (WIDE) bf16 GEMM tiles for dZ and the weight gradients: bf16-GEMM / C5 / long-key /
# headline parity, C5 A/B against 128 x 128 (MMF_GEMM_NO_WIDE=1), traffic of both.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05aa}
mkdir -p $O
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 500 $PT tests/test_gpu_gemm_bf16.py tests/test_gpu_c5_bench.py tests/test_gpu_bf16.py tests/test_gpu_train_mode.py tests/test_gpu_headline.py > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
B="python bench.py --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu"
for i in 1 2; do
  timeout -k 10 200 $B > $O/c5_wide$i.json 2> $O/c5_wide$i.err || exit $?
  timeout -k 10 200 env MMF_GEMM_NO_WIDE=1 $B > $O/c5_narrow$i.json 2> $O/c5_narrow$i.err || exit $?
done
PB="python3 bench.py --workload c5 --precision medium --steps 2 --warmup 1 --skip-cpu --no-graph --profile-steps 1"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d /tmp/pf -o run -- $PB > $O/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d /tmp/pw -o run -- $PB > $O/pmc_write.log 2>&1 || exit 1
python3 profiles/pmc_traffic.py /tmp/pf/run_counter_collection.csv /tmp/pw/run_counter_collection.csv "r05aa c5 medium: $PB" $O/pmc_traffic_c5_medium.json || exit 1
echo done
