#!/bin/bash
# Headline c2 parity alone and behind the train-step tests (order check, with the diff report);
# then the long-key attention phase stamps (backward, forward) from libmmfusion_stampsl.so.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05t}
mkdir -p $O
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu"
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 200 $PT tests/test_gpu_headline.py > $O/headline_alone.log 2>&1; rc=$?; echo "headline alone rc=$rc"; fatal $rc alone
timeout -k 10 400 $PT tests/test_gpu_train_step.py tests/test_gpu_headline.py > $O/order.log 2>&1; rc=$?; echo "order rc=$rc"; fatal $rc order
SL=multimodal-sensor-fusion-with-attention-rajeevatla_amd/csrc/libmmfusion_stampsl.so
timeout -k 10 200 env MMF_LIB_PATH=$SL python scripts/attn_stamps.py long > $O/stamps_long.json 2> $O/stamps_long.err || exit $?
timeout -k 10 200 env MMF_LIB_PATH=$SL python scripts/attn_stamps.py longf > $O/stamps_longf.json 2> $O/stamps_longf.err || exit $?
echo done
