# A/B of the GEMM group interleave (MMF_GEMM_ILV): bit-exactness test, then C5 (medium) and
# C2 bench lines with it off and on.  usage: bash scripts/gpu_ilv_ab.sh <run-name>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
RUN=${1:-ilv}
O=gpurun_out/$RUN
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_train_mode.py -k interleave > $O/pytest.log 2>&1 || exit 1
echo "test ok"
for ilv in 0 1; do
  for wp in c5:medium c5:highest c2:highest; do
    wl=${wp%%:*}; pr=${wp##*:}
    MMF_GEMM_ILV=$ilv timeout -k 10 300 python -u bench.py --workload $wl --precision $pr --steps 20 --warmup 5 --skip-cpu > $O/${wl}_${pr}_ilv${ilv}.json 2> $O/${wl}_${pr}_ilv${ilv}.err || exit 1
    echo "$wl $pr ilv=$ilv ok"
  done
done
echo done
