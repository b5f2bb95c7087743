#!/bin/bash
# Eager L = 1 step through bench.py's default policy (replay_pays): train-step / headline / C-ABI
# GPU tests, then the c2_l1 bench line with its rocprofv3 kernel stats, twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05s}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_train_step.py tests/test_gpu_headline.py tests/test_capi_abi.py > $O/pytest.log 2>&1 || exit $?
bash scripts/gpu_prof.sh $O c2_l1 --workload c2_l1 --steps 500 --warmup 50 || exit $?
timeout -k 10 200 python bench.py --workload c2_l1 --steps 500 --warmup 50 --skip-cpu > $O/l1_default2.json 2> $O/l1_default2.err || exit $?
echo done
