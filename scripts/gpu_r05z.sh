#!/bin/bash
# C5 medium A/B after the prefetch fix: the 8-wave long forward (MMF_LONG_FWD_W8=1) against the
# 16-wave product, and the keep words drawn serially on the main stream (MMF_KW_SERIAL=1: what the
# side-stream overlap saves or costs the concurrent GEMMs); libmmfusion_pk.so: the exp arguments
# as packed FMAs in both long kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05z}
mkdir -p $O
B="python bench.py --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu"
for i in 1 2; do
  timeout -k 10 200 $B > $O/c5_w16_$i.json 2> $O/c5_w16_$i.err || exit $?
  timeout -k 10 200 env MMF_LONG_FWD_W8=1 $B > $O/c5_w8_$i.json 2> $O/c5_w8_$i.err || exit $?
  timeout -k 10 200 env MMF_LIB_PATH=multimodal-sensor-fusion-with-attention-rajeevatla_amd/csrc/libmmfusion_pk.so $B > $O/c5_pk_$i.json 2> $O/c5_pk_$i.err || exit $?
done
timeout -k 10 200 env MMF_KW_SERIAL=1 $B > $O/c5_kwserial.json 2> $O/c5_kwserial.err || exit $?
echo done
