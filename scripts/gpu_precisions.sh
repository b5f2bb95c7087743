# GPU tests, then the C2 bench line at each matmul precision (top kernels).
# usage (on the box): bash scripts/gpu_precisions.sh <run-name> [bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
RUN=${1:-prec}; shift
O=gpurun_out/$RUN
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log; tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^E |Error|assert" $O/pytest_gpu.log | head -30; exit $rc; fi
for pr in highest high medium; do
  timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --skip-cpu --precision $pr "$@" > $O/bench_$pr.json 2> $O/bench_$pr.err || exit 1
  python3 -c "import json;d=json.load(open('$O/bench_$pr.json'));print('$pr', d['ms_per_step'], d['value'], d['dtype']);[print('   %-44s %8.1f us  %s %.3f' % (k[:44], v['avg_launch_ms']*1e3, v['bound'], v['frac'])) for k,v in list(d['kernels'].items())[:8]]"
done
