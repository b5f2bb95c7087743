# Keep words drawn inside the input-mask kernel (MMF_KW_FUSED=1): GPU tests with the default plan
# and with the switch, then same-box A/B lines on C2 and C5 "medium".
# usage: bash scripts/gpu_kw_fused.sh <run-name>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-kwf}
mkdir -p $O
[ -n "$SKIP_FULL" ] || timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
MMF_KW_FUSED=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_train_mode.py tests/test_gpu_bf16.py -k "not side_stream" -x -q --timeout 120 --timeout-method thread > $O/pytest_fused.log 2>&1 || { tail -30 $O/pytest_fused.log; exit 1; }
tail -1 $O/pytest_fused.log
bash scripts/gpu_env_ab.sh ${1:-kwf} default fused serial || exit 1
WORKLOAD=c5 PRECISION=medium STEPS=20 bash scripts/gpu_env_ab.sh ${1:-kwf} default fused || exit 1
echo all done
