#!/bin/bash
# Iteration check: every GPU test, the L1 stamps, the C2-L1 and C2 lines with kernel stats (no CPU legs).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-iter}
mkdir -p $O
P=multimodal-sensor-fusion-with-attention-rajeevatla_amd/csrc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 120 env MMF_LIB_PATH=$P/libmmfusion_stampsl1.so python scripts/l1_stamps.py > $O/l1_stamps.json 2> $O/l1_stamps.err || exit $?
bash scripts/gpu_prof.sh $O c2_l1 --workload c2_l1 --steps 100 --warmup 20 --skip-cpu || exit $?
bash scripts/gpu_prof.sh $O c2 --steps 50 --warmup 10 --skip-cpu || exit $?
echo done
