#!/bin/bash
# Poisoned-allocator step test (c2, c2_l1); the train-step -> headline order again; C5 medium
# A/B/C: product (bwd Q-image store before barrier B + dQ offsets hoisted + forward loads two
# blocks ahead), libmmfusion_ab.so (attn_long.hip at HEAD), libmmfusion_prio.so (product +
# s_setprio 1 for the younger half), libmmfusion_dbuf.so (product + scores double-buffered by a
# two-way unrolled loop); stamps at the product.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05v}
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 300 $PT tests/test_gpu_headline.py -k uninitialized > $O/poison.log 2>&1; rc=$?; echo "poison rc=$rc"; fatal $rc poison
timeout -k 10 400 $PT tests/test_gpu_train_step.py tests/test_gpu_headline.py > $O/order.log 2>&1; rc=$?; echo "order rc=$rc"; fatal $rc order
timeout -k 10 300 $PT tests/test_gpu_c5_bench.py tests/test_gpu_bf16.py > $O/parity_long.log 2>&1 || exit $?
P=multimodal-sensor-fusion-with-attention-rajeevatla_amd/csrc
for i in 1 2; do
  for V in new ab prio dbuf; do
    L=""; [ $V != new ] && L="MMF_LIB_PATH=$P/libmmfusion_$V.so"
    timeout -k 10 200 env $L python bench.py --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu > $O/c5_$V$i.json 2> $O/c5_$V$i.err || exit $?
  done
done
timeout -k 10 200 env MMF_LIB_PATH=$P/libmmfusion_stampsl.so python scripts/attn_stamps.py long > $O/stamps_long.json 2> $O/stamps_long.err || exit $?
timeout -k 10 200 env MMF_LIB_PATH=$P/libmmfusion_stampsl.so python scripts/attn_stamps.py longf > $O/stamps_longf.json 2> $O/stamps_longf.err || exit $?
echo done
