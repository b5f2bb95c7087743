#!/bin/bash
# Round-4 close evidence in one GPU call: every GPU test, smoke, the C2 line (CPU legs) with its
# rocprofv3 stats, PMC FETCH/WRITE passes for C2 and C2-L1, the C2-L1 line (CPU legs) with stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
RUN=${1:-close}
O=gpurun_out/$RUN
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed rc=$rc"; exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
for WL in c2 c2_l1; do
  PB="python3 bench.py --workload $WL --steps 2 --warmup 1 --skip-cpu --no-graph --profile-steps 1"
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d /tmp/pf_$WL -o run -- $PB > $O/pmc_fetch_$WL.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d /tmp/pw_$WL -o run -- $PB > $O/pmc_write_$WL.log 2>&1 || exit 1
  python3 profiles/pmc_traffic.py /tmp/pf_$WL/run_counter_collection.csv /tmp/pw_$WL/run_counter_collection.csv "$RUN: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over: $PB" $O/pmc_traffic_$WL.json || exit 1
  rm -rf /tmp/pf_$WL /tmp/pw_$WL
done
cp $O/pmc_traffic_c2.json profiles/pmc_traffic.json
cp $O/pmc_traffic_c2_l1.json profiles/pmc_traffic_c2_l1_highest.json
bash scripts/gpu_prof.sh $O c2 --steps 50 --warmup 10 || exit $?
bash scripts/gpu_prof.sh $O c2_l1 --workload c2_l1 --steps 100 --warmup 20 || exit $?
echo closed
