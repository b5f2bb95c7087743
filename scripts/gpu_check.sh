# One GPU call closing a state of the tree: the whole -m gpu suite, smoke(), PMC traffic and SQ
# passes over C2, the driver's bench command (and the default one), its rocprofv3 kernel stats.
# usage (on the box): bash scripts/gpu_check.sh <run-name>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
RUN=${1:-r1}
O=gpurun_out/$RUN
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
[ $rc -ne 0 ] && { echo "gpu suite failed rc=$rc"; tail -40 $O/pytest_gpu.log; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
# HBM traffic: FETCH_SIZE and WRITE_SIZE in passes of their own (4 TCC slots), kernel-trace only
PB="python3 bench.py --steps 2 --warmup 1 --skip-cpu --no-graph --profile-steps 1"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- $PB > $O/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- $PB > $O/pmc_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
python3 profiles/pmc_traffic.py $O/pmc_fetch/run_counter_collection.csv $O/pmc_write/run_counter_collection.csv "$RUN: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over: $PB" $O/pmc_traffic.json || exit 1
cp $O/pmc_traffic.json profiles/pmc_traffic.json
bash profiles/collect_pmc.sh $O/pmc_sq_c2 > $O/pmc_sq.log 2>&1 || { echo "sq passes failed"; exit 1; }
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit 1
timeout -k 10 300 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --skip-cpu > $O/prof_bench.json 2> $O/prof.err || exit 1
echo done
