# GPU tests of the long-key / GEMM paths, then C5 (medium) and C2 bench lines.
# usage: bash scripts/gpu_r03c.sh <run-name>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
RUN=${1:-r03c}
O=gpurun_out/$RUN
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_bf16.py tests/test_gpu_train_mode.py > $O/pytest.log 2>&1 || { echo "pytest failed"; exit 1; }
echo "tests ok"
for wp in c5:medium c2:highest; do
  wl=${wp%%:*}; pr=${wp##*:}
  timeout -k 10 300 python -u bench.py --workload $wl --precision $pr --steps 20 --warmup 5 --skip-cpu > $O/${wl}_${pr}.json 2> $O/${wl}_${pr}.err || exit 1
  echo "$wl $pr ok"
done
echo done
