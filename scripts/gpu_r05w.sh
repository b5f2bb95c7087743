#!/bin/bash
# Long-key attention prefetches as buffer loads with no use until the consumer (the per-block
# global round trips off the critical path) + s_setprio for the younger half: parity of the long
# kernels, C5 medium A/B/C (product, attn_long.hip at 40c2e52, product without the setprio),
# phase stamps, and the C2 seed sweep against the oracle.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05w}
mkdir -p $O
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 400 $PT tests/test_gpu_c5_bench.py tests/test_gpu_bf16.py tests/test_gpu_train_mode.py tests/test_gpu_parity.py > $O/parity_long.log 2>&1 || exit $?
P=multimodal-sensor-fusion-with-attention-rajeevatla_amd/csrc
for i in 1 2; do
  for V in new ab noprio; do
    L=""; [ $V != new ] && L="MMF_LIB_PATH=$P/libmmfusion_$V.so"
    timeout -k 10 200 env $L python bench.py --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu > $O/c5_$V$i.json 2> $O/c5_$V$i.err || exit $?
  done
done
timeout -k 10 200 env MMF_LIB_PATH=$P/libmmfusion_stampsl.so python scripts/attn_stamps.py long > $O/stamps_long.json 2> $O/stamps_long.err || exit $?
timeout -k 10 200 env MMF_LIB_PATH=$P/libmmfusion_stampsl.so python scripts/attn_stamps.py longf > $O/stamps_longf.json 2> $O/stamps_longf.err || exit $?
timeout -k 10 300 python scripts/seed_sweep.py --seeds 6 > $O/seed_sweep.txt 2> $O/seed_sweep.err || exit $?
echo done
