#!/bin/bash
# Full GPU suite at the work tree, then: C5 4-deep bf16 ring A/B (MMF_GEMM_B16_NS4=1) and the
# C2-L1 step with the clip + AdamW operand prefetch (product) against HEAD's head.hip (libmmfusion_base.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05aj}
mkdir -p $O
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
L1="python bench.py --workload c2_l1 --steps 500 --warmup 50 --skip-cpu"
BASE=multimodal-sensor-fusion-with-attention-rajeevatla_amd/csrc/libmmfusion_base.so
for i in 1 2; do
  timeout -k 10 120 $L1 > $O/l1_pf_$i.json 2> $O/l1_pf_$i.err || exit $?
  timeout -k 10 120 env MMF_LIB_PATH=$BASE $L1 > $O/l1_base_$i.json 2> $O/l1_base_$i.err || exit $?
done
B="python bench.py --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu"
for i in 1 2; do
  timeout -k 10 200 $B > $O/c5_ns3_$i.json 2> $O/c5_ns3_$i.err || exit $?
  timeout -k 10 200 env MMF_GEMM_B16_NS4=1 $B > $O/c5_ns4_$i.json 2> $O/c5_ns4_$i.err || exit $?
done
echo done
