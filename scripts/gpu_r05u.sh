#!/bin/bash
# (1) which train-step test leaves the state that fails headline[c2] (one pytest process per
# test function, then headline c2); (2) long-key attention parity at the head; (3) C5 medium
# A/B: product lib (bwd Q-image store before barrier B, dQ store offsets hoisted) against
# libmmfusion_ab.so (attn_long.hip at HEAD), alternating; (4) stamps at the head.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05u}
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
for F in test_clip_and_adamw_match_torch test_graph_follows_lr_and_new_batches test_load_batch_rejects_new_shapes \
         test_fused_clip_adamw_matches_two_call_path test_gradient_accumulation_equals_full_batch \
         test_accumulate_rejects_uneven_micro_batches test_one_call_train_step_matches_three_calls \
         test_clip_partials_from_the_train_step test_tile_head_train_step \
         test_tile_head_module_path_matches_per_sample_head test_l1_poll_timeout_surfaces_and_recovers; do
  timeout -k 10 200 $PT tests/test_gpu_train_step.py -k $F "tests/test_gpu_headline.py::test_benchmark_step_matches_oracle[c2]" > $O/bisect_$F.log 2>&1; rc=$?
  echo "bisect $F rc=$rc" | tee -a $O/bisect.txt; fatal $rc $F
done
timeout -k 10 400 $PT tests/test_gpu_c5_bench.py tests/test_gpu_bf16.py tests/test_gpu_train_mode.py tests/test_gpu_parity.py > $O/parity.log 2>&1 || exit $?
P=multimodal-sensor-fusion-with-attention-rajeevatla_amd/csrc
for i in 1 2; do
  timeout -k 10 200 python bench.py --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu > $O/c5_new$i.json 2> $O/c5_new$i.err || exit $?
  timeout -k 10 200 env MMF_LIB_PATH=$P/libmmfusion_ab.so python bench.py --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu > $O/c5_old$i.json 2> $O/c5_old$i.err || exit $?
done
timeout -k 10 200 env MMF_LIB_PATH=$P/libmmfusion_stampsl.so python scripts/attn_stamps.py long > $O/stamps_long.json 2> $O/stamps_long.err || exit $?
timeout -k 10 200 env MMF_LIB_PATH=$P/libmmfusion_stampsl.so python scripts/attn_stamps.py longf > $O/stamps_longf.json 2> $O/stamps_longf.err || exit $?
echo done
