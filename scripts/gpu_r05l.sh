#!/bin/bash
# XCD-aware GEMM tile order: every GPU test, the C5 line + its traffic, the C2 line (unchanged tile
# order there) and C4.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05l}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed rc=$rc"; exit $rc; fi
grep -q "illegal memory access\|Memory access fault" $O/pytest_gpu.log && { echo "GPU fault: stopping"; exit 1; }
bash scripts/gpu_prof.sh $O c5_medium --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu || exit $?
PB="python3 bench.py --workload c5 --precision medium --steps 2 --warmup 1 --skip-cpu --no-graph --profile-steps 1"
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d /tmp/pf -o run -- $PB > $O/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d /tmp/pw -o run -- $PB > $O/pmc_write.log 2>&1 || exit 1
python3 profiles/pmc_traffic.py /tmp/pf/run_counter_collection.csv /tmp/pw/run_counter_collection.csv "r05l c5 medium: $PB" $O/pmc_traffic_c5_medium.json || exit 1
bash scripts/gpu_prof.sh $O c2 --steps 100 --warmup 20 || exit $?
timeout -k 10 300 python bench.py --workload c4 --precision medium --steps 20 --warmup 5 --skip-cpu > $O/c4_medium.json 2> $O/c4_medium.err || exit $?
echo done
