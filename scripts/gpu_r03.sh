# Round-3 iteration: GPU tests, then bench lines for the listed workloads (no profiling passes).
# usage: bash scripts/gpu_r03.sh <run-name> <workload[:extra-args]>...   e.g. c2 c2_l1 "c2:--path module"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
RUN=${1:-q}; shift
O=gpurun_out/$RUN
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  # failures are read afterwards; a crash (rc other than 0 / 1) ends the call
  timeout -k 10 500 python -u -m pytest tests -m gpu --maxfail=8 -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log; tail -3 $O/pytest_gpu.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
i=0
for spec0 in "$@"; do
  # spec: workload[:bench args][@VAR=VAL] (one environment assignment for the run)
  spec=${spec0%%@*}; envset=""
  [ "$spec0" != "$spec" ] && envset=${spec0#*@}
  wl=${spec%%:*}; extra=""
  [ "$spec" != "$wl" ] && extra=${spec#*:}
  i=$((i+1))
  env $envset timeout -k 10 300 python -u bench.py --workload $wl --steps 50 --warmup 10 --skip-cpu $extra > $O/bench_${i}_$wl.json 2> $O/bench_${i}_$wl.err || exit 1
  python3 -c "import json;d=json.load(open('$O/bench_${i}_$wl.json'));print('$spec0', d['ms_per_step'], d.get('ms_per_step_median'), d['value']);print(json.dumps(d['kernels'],indent=0)[:1500])"
done
