# Long-key kernel VALU trims + GEMM interleave: GPU tests of the touched paths, then bench
# lines with the interleave off / on.  usage: bash scripts/gpu_r03b.sh <run-name>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
RUN=${1:-r03b}
O=gpurun_out/$RUN
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_bf16.py tests/test_gpu_train_mode.py > $O/pytest.log 2>&1 || { echo "pytest failed"; exit 1; }
echo "tests ok"
for ilv in 0 1; do
  for wp in c5:medium c2:highest; do
    wl=${wp%%:*}; pr=${wp##*:}
    MMF_GEMM_ILV=$ilv timeout -k 10 300 python -u bench.py --workload $wl --precision $pr --steps 20 --warmup 5 --skip-cpu > $O/${wl}_${pr}_ilv${ilv}.json 2> $O/${wl}_${pr}_ilv${ilv}.err || exit 1
    echo "$wl $pr ilv=$ilv ok"
  done
done
echo done
