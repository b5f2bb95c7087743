#!/bin/bash
# Round-close C5 evidence in one GPU call: the C5 bench line (medium, with its CPU baseline),
# rocprofv3 kernel stats of the same command, PMC traffic passes, SQ counter passes.
# usage (on the box): bash scripts/gpu_close_c5.sh <run-name>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
RUN=${1:-close_c5}
O=gpurun_out/$RUN
mkdir -p $O
W="--workload c5 --precision medium"
timeout -k 10 300 python -u bench.py $W --steps 20 --warmup 5 > $O/bench_c5.json 2> $O/bench_c5.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py $W --steps 20 --warmup 5 --skip-cpu > $O/prof_bench_c5.json 2> $O/prof.err || exit 1
PB="python3 bench.py --steps 2 --warmup 1 --skip-cpu --no-graph --profile-steps 1 $W"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- $PB > $O/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- $PB > $O/pmc_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
python3 profiles/pmc_traffic.py $O/pmc_fetch/run_counter_collection.csv $O/pmc_write/run_counter_collection.csv "$RUN: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over: $PB" $O/pmc_traffic_c5.json || exit 1
bash profiles/collect_pmc.sh $O/sq $W || exit 1
echo closed
