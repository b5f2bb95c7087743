# A/B on the box: GPU parity tests, then the bench once per environment setting.
# usage: bash scripts/gpu_ab.sh <run-name> "<ENV=VAL ...>" ["<ENV=VAL ...>" ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
RUN=${1:-ab}; shift
O=gpurun_out/$RUN
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log; tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
i=0
for E in "$@"; do
  i=$((i+1))
  env $E timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --skip-cpu > $O/bench_$i.json 2> $O/bench_$i.err || exit 1
  python3 -c "import json;d=json.load(open('$O/bench_$i.json'));print('$E', d['ms_per_step'], d['value']);[print('  ',k,v['avg_launch_ms'],v['frac']) for k,v in list(d['kernels'].items())[:6]]"
done
