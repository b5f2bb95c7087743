#!/bin/bash
# C5 "medium" at the head: parity tests, the pool_e A/B, the HBM traffic passes and the SQ passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05k}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_c5_bench.py tests/test_gpu_bf16.py tests/test_gpu_train_mode.py tests/test_gpu_gemm_bf16.py -v --timeout 300 --timeout-method thread > $O/pytest_medium.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_medium.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed rc=$rc"; exit $rc; fi
grep -q "illegal memory access\|Memory access fault" $O/pytest_medium.log && { echo "GPU fault: stopping"; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu > $O/c5_a$i.json 2> $O/c5_a$i.err || exit $?
  MMF_POOLE_FLAT=1 timeout -k 10 300 python bench.py --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu > $O/c5_b$i.json 2> $O/c5_b$i.err || exit $?
done
PB="python3 bench.py --workload c5 --precision medium --steps 2 --warmup 1 --skip-cpu --no-graph --profile-steps 1"
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d /tmp/pf -o run -- $PB > $O/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d /tmp/pw -o run -- $PB > $O/pmc_write.log 2>&1 || exit 1
python3 profiles/pmc_traffic.py /tmp/pf/run_counter_collection.csv /tmp/pw/run_counter_collection.csv "r05k c5 medium: $PB" $O/pmc_traffic_c5_medium.json || exit 1
timeout -k 10 400 bash profiles/collect_pmc.sh $O/pmc_c5 --workload c5 --precision medium > $O/pmc_c5.log 2>&1 || exit $?
rm -rf $O/pmc_c5/p1 $O/pmc_c5/p2 $O/pmc_c5/p3
echo done
