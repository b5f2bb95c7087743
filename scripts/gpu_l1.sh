#!/bin/bash
# L1 iteration: the train-step / single-key / headline GPU tests, L1 stamps, the C2-L1 line + kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-l1}
mkdir -p $O
P=multimodal-sensor-fusion-with-attention-rajeevatla_amd/csrc
timeout -k 10 300 python -u -m pytest tests/test_gpu_train_step.py tests/test_gpu_single_key.py tests/test_gpu_headline.py -x -q --timeout 120 --timeout-method thread > $O/pytest_l1.log 2>&1 || exit $?
timeout -k 10 120 env MMF_LIB_PATH=$P/libmmfusion_stampsl1.so python scripts/l1_stamps.py > $O/l1_stamps.json 2> $O/l1_stamps.err || exit $?
bash scripts/gpu_prof.sh $O c2_l1 --workload c2_l1 --steps 100 --warmup 20 --skip-cpu || exit $?
echo done
