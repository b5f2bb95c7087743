# Pipelined lean forward: GPU tests (default = pipelined), the many-item train case at p = 0,
# then C2 bench A/B against the one-item kernel (MMF_FWD_PIPE=0), alternating arms.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-pipe}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log; tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
DIAG_P=0 timeout -k 10 300 python -u scripts/diag_train_case.py train_pipe highest > $O/diag_highest_p0.txt 2>&1 || exit 1
DIAG_P=0 timeout -k 10 300 python -u scripts/diag_train_case.py train_pipe high > $O/diag_high_p0.txt 2>&1 || exit 1
for arm in 1 0 1 0; do
  MMF_FWD_PIPE=$arm timeout -k 10 300 python -u bench.py --skip-cpu --steps 100 > $O/bench_$arm.json 2>> $O/bench.err || exit 1
  cat $O/bench_$arm.json >> $O/bench_all.jsonl
done
echo done
