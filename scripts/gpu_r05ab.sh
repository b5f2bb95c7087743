#!/bin/bash
# C5 A/B: Q-image staging and the LSE / D stores moved to the younger half of the long-key
# attention workgroups (libmmfusion_bal.so) against the product; long-key parity with it.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05ab}
mkdir -p $O
L=multimodal-sensor-fusion-with-attention-rajeevatla_amd/csrc/libmmfusion_bal.so
timeout -k 10 400 env MMF_LIB_PATH=$L python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_c5_bench.py tests/test_gpu_bf16.py tests/test_gpu_train_mode.py > $O/pytest_bal.log 2>&1 || exit $?
B="python bench.py --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu"
for i in 1 2; do
  timeout -k 10 200 $B > $O/c5_prod$i.json 2> $O/c5_prod$i.err || exit $?
  timeout -k 10 200 env MMF_LIB_PATH=$L $B > $O/c5_bal$i.json 2> $O/c5_bal$i.err || exit $?
done
echo done
