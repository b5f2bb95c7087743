# Round-3 close evidence at the session head in one GPU call: GPU tests, the C2 headline bench
# line (with the CPU legs), its kernel stats / HBM traffic / SQ passes, the C2 L = 1 line + stats,
# and the C5 "medium" line + stats / traffic / SQ passes.  usage: bash scripts/gpu_close_r03b.sh <run>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
RUN=${1:-close3b}
O=gpurun_out/$RUN
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log; tail -2 $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || exit 1
echo "bench ok"
bash scripts/gpu_profile_r03.sh $RUN/c2 || exit 1
timeout -k 10 300 python -u bench.py --workload c2_l1 --skip-cpu > $O/bench_c2_l1.json 2> $O/bench_c2_l1.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2_l1_prof -o run -- \
  python3 bench.py --workload c2_l1 --steps 30 --warmup 5 --skip-cpu > $O/c2_l1_prof_bench.json 2> $O/c2_l1_prof.err || exit 1
echo "c2_l1 ok"
timeout -k 10 300 python -u bench.py --workload c5 --precision medium --skip-cpu > $O/bench_c5m.json 2> $O/bench_c5m.err || exit 1
bash scripts/gpu_profile_r03.sh $RUN/c5m --workload c5 --precision medium || exit 1
echo closed
