#!/bin/bash
# C5 iteration: the bf16 / train-mode GPU tests, then the C5 "medium" line + kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
RUN=${1:-c5b}
O=gpurun_out/$RUN
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_train_mode.py -x -q --timeout 120 --timeout-method thread > $O/pytest_c5.log 2>&1 || exit $?
bash scripts/gpu_c5.sh $RUN || exit $?
echo done
