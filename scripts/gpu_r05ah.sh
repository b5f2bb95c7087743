#!/bin/bash
# C5: weight-gradient split-K cap A/B (MMF_WGRAD_SPLIT_CAP: fewer slabs, less reduce traffic)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05ah}
mkdir -p $O
B="python bench.py --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu"
for i in 1 2; do
  timeout -k 10 200 $B > $O/c5_def_$i.json 2> $O/c5_def_$i.err || exit $?
  for c in 8 16 24; do
    timeout -k 10 200 env MMF_WGRAD_SPLIT_CAP=$c $B > $O/c5_cap${c}_$i.json 2> $O/c5_cap${c}_$i.err || exit $?
  done
done
echo done
