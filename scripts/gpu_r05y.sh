#!/bin/bash
# fp32-MFMA grouped pools (U with padded pbar rows, dpbar, E): C5 / long-key / pooled parity, the
# headline order check, C5 A/B against the VALU forms (MMF_POOL_VALU=1), rocprofv3 stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05y}
mkdir -p $O
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 500 $PT tests/test_gpu_c5_bench.py tests/test_gpu_bf16.py tests/test_gpu_train_mode.py tests/test_gpu_parity.py tests/test_gpu_train_step.py tests/test_gpu_headline.py > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
for i in 1 2; do
  timeout -k 10 200 python bench.py --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu > $O/c5_mfma$i.json 2> $O/c5_mfma$i.err || exit $?
  timeout -k 10 200 env MMF_POOL_VALU=1 python bench.py --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu > $O/c5_valu$i.json 2> $O/c5_valu$i.err || exit $?
done
bash scripts/gpu_prof.sh $O c5_medium --workload c5 --precision medium --steps 20 --warmup 5 || exit $?
echo done
