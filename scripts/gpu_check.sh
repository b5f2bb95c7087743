set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
RUN=${1:-r1}
mkdir -p gpurun_out/$RUN
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$RUN/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/$RUN/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed rc=$rc"; exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 > gpurun_out/$RUN/bench.json 2> gpurun_out/$RUN/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$RUN/prof -o run -- python3 bench.py --steps 20 --warmup 5 --skip-cpu > gpurun_out/$RUN/prof_bench.json 2> gpurun_out/$RUN/prof.err
echo done
