#!/bin/bash
# L1 stamps + launch micro-benchmark + module / compiled paths after the set-to-none gradients.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r04b}
mkdir -p $O
P=multimodal-sensor-fusion-with-attention-rajeevatla_amd/csrc
timeout -k 10 120 env MMF_LIB_PATH=$P/libmmfusion_stampsl1.so python scripts/l1_stamps.py > $O/l1_stamps.json 2> $O/l1_stamps.err || exit $?
timeout -k 10 120 scripts/micro/launch_micro > $O/launch_micro.txt 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_compile.py tests/test_dp.py tests/test_gpu_train_step.py -x -q --timeout 120 --timeout-method thread > $O/pytest_sub.log 2>&1 || exit $?
bash scripts/gpu_paths.sh $O c2 || exit $?
echo done
