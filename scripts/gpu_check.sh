# One GPU call: parity tests, PMC traffic passes, bench, rocprofv3 kernel stats.
# usage (on the box): bash scripts/gpu_check.sh <run-name>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
RUN=${1:-r1}
O=gpurun_out/$RUN
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed rc=$rc"; exit $rc; fi
# HBM traffic: FETCH_SIZE and WRITE_SIZE in passes of their own (4 TCC slots), kernel-trace only
PB="python3 bench.py --steps 2 --warmup 1 --skip-cpu --no-graph --profile-steps 1"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- $PB > $O/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- $PB > $O/pmc_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
python3 profiles/pmc_traffic.py $O/pmc_fetch/run_counter_collection.csv $O/pmc_write/run_counter_collection.csv "$RUN: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over: $PB" $O/pmc_traffic.json || exit 1
cp $O/pmc_traffic.json profiles/pmc_traffic.json
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 50 --warmup 10 --skip-cpu > $O/prof_bench.json 2> $O/prof.err
echo done
