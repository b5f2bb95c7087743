# Session re-entry check: GPU tests, the C2 headline line, C5 medium line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-s1}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log; tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --skip-cpu > $O/bench_c2.json 2> $O/bench_c2.err || exit 1
timeout -k 10 300 python -u bench.py --workload c5 --precision medium --skip-cpu > $O/bench_c5m.json 2> $O/bench_c5m.err || exit 1
timeout -k 10 200 python -u scripts/lib_gemm_ceiling.py > $O/lib_gemm.json 2> $O/lib_gemm.err || exit 1
echo done
