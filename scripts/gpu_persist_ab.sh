# Persistent fused backward: GPU tests, then C2 bench A/B against the one-item grid
# (MMF_FUSED_PERSIST=0), alternating arms; C5 medium and C4 lines per arm.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-persist}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log; tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
for arm in 1 0 1 0; do
  MMF_FUSED_PERSIST=$arm timeout -k 10 300 python -u bench.py --skip-cpu --steps 100 > $O/bench_$arm.json 2>> $O/bench.err || exit 1
  cat $O/bench_$arm.json >> $O/bench_all.jsonl
done
for arm in 1 0; do
  MMF_FUSED_PERSIST=$arm timeout -k 10 300 python -u bench.py --skip-cpu --workload c4 > $O/bench_c4_$arm.json 2>> $O/bench.err || exit 1
done
echo done
