# Iteration loop on the box: GPU parity tests, then one bench line (no profiling passes).
# usage: bash scripts/gpu_quick.sh <run-name> [bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
RUN=${1:-q}; shift
O=gpurun_out/$RUN
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log; tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --skip-cpu "$@" > $O/bench.json 2> $O/bench.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['ms_per_step'], d['value']);print(json.dumps(d['kernels'],indent=0))"
