# Round-3 profiles for one workload in one GPU call (no tests): rocprofv3 kernel stats of the
# bench command, the HBM traffic passes (FETCH_SIZE, WRITE_SIZE) and the SQ counter passes.
# usage (on the box): bash scripts/gpu_profile_r03.sh <run-name> [extra bench.py args]
#   e.g. bash scripts/gpu_profile_r03.sh p_c2      |  bash scripts/gpu_profile_r03.sh p_c5 --workload c5 --precision medium
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
RUN=${1:-prof}; shift
O=gpurun_out/$RUN
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 30 --warmup 5 --skip-cpu "$@" > $O/prof_bench.json 2> $O/prof.err || { echo "stats failed"; exit 1; }
echo "stats ok"
PB="python3 bench.py --steps 2 --warmup 1 --skip-cpu --no-graph --profile-steps 1 $*"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- $PB > $O/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- $PB > $O/pmc_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
python3 profiles/pmc_traffic.py $O/pmc_fetch/run_counter_collection.csv $O/pmc_write/run_counter_collection.csv "$RUN: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over: $PB" $O/pmc_traffic.json || exit 1
echo "traffic ok"
bash profiles/collect_pmc.sh $O/sq "$@" || exit 1
echo "profiled"
