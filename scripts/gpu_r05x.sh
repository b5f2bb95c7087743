#!/bin/bash
# Head checks after the long-key prefetch fix and the fp32-MFMA grouped pools: the whole GPU suite,
# the C5 medium line (with its CPU baseline) + rocprofv3 stats, the pools A/B (MMF_POOL_VALU=1: the
# VALU forms), C5 traffic and SQ passes, the C2 seed sweep with the ReLU slack.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05x}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
case $rc in 124|134|137|139) echo "pytest crashed rc=$rc"; exit $rc;; esac
bash scripts/gpu_prof.sh $O c5_medium --workload c5 --precision medium --steps 20 --warmup 5 || exit $?
for i in 1 2; do
  timeout -k 10 200 python bench.py --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu > $O/c5_mfma$i.json 2> $O/c5_mfma$i.err || exit $?
  timeout -k 10 200 env MMF_POOL_VALU=1 python bench.py --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu > $O/c5_valu$i.json 2> $O/c5_valu$i.err || exit $?
done
PB="python3 bench.py --workload c5 --precision medium --steps 2 --warmup 1 --skip-cpu --no-graph --profile-steps 1"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d /tmp/pf -o run -- $PB > $O/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d /tmp/pw -o run -- $PB > $O/pmc_write.log 2>&1 || exit 1
python3 profiles/pmc_traffic.py /tmp/pf/run_counter_collection.csv /tmp/pw/run_counter_collection.csv "r05x c5 medium: $PB" $O/pmc_traffic_c5_medium.json || exit 1
bash profiles/collect_pmc.sh /tmp/sq_c5 --workload c5 --precision medium > $O/sq_c5.log 2>&1 || exit 1
cp /tmp/sq_c5/pmc_summary.json $O/pmc_sq_c5_medium.json
python3 profiles/pmc_summary.py /tmp/sq_c5 $O/pmc_sq_c5_medium.json > $O/pmc_sq_c5_medium.txt 2>&1 || true
timeout -k 10 300 python scripts/seed_sweep.py --seeds 4 > $O/seed_sweep.txt 2> $O/seed_sweep.err || exit $?
echo done
