#!/bin/bash
# C5 check: every GPU test, then the C5 "medium" line + kernel stats.  usage: bash scripts/gpu_c5t.sh <run>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
RUN=${1:-c5t}
O=gpurun_out/$RUN
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
bash scripts/gpu_prof.sh $O c5_medium --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu || exit $?
echo done
