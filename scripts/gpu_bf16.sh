# bf16 math-mode check on the box: GPU tests, then C2 / C5 bench lines at both precisions.
# usage: bash scripts/gpu_bf16.sh <run-name>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
RUN=${1:-bf}
O=gpurun_out/$RUN
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log; tail -5 $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for cfg in "c2 highest 50 10" "c2 medium 50 10" "c5 highest 6 2" "c5 medium 10 3"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --workload $1 --precision $2 --steps $3 --warmup $4 --skip-cpu > $O/bench_$1_$2.json 2> $O/bench_$1_$2.err || exit 1
  python3 -c "import json;d=json.load(open('$O/bench_$1_$2.json'));print('$1 $2', d['ms_per_step'], d['value']);[print('  ',k,v['ms_per_step'],v['achieved'],v['frac']) for k,v in list(d['kernels'].items())[:8]]"
done
exit $rc
