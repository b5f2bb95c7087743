#!/bin/bash
# C5 "medium" (bf16) line + kernel stats + launch dump.  usage: bash scripts/gpu_c5.sh <run> [extra bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
RUN=${1:-c5}; shift
O=gpurun_out/$RUN
mkdir -p $O
bash scripts/gpu_prof.sh $O c5_medium --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu --dump-launches $O/c5_launches.json "$@" || exit $?
echo done
