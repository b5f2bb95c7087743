#!/bin/bash
# Round-close evidence, both workloads, one GPU call: scripts/gpu_roundclose.sh (full GPU suite,
# C2 traffic / bench / rocprof / SQ) then scripts/gpu_close_c5.sh (C5 bench / rocprof / traffic / SQ).
set -o pipefail
cd $GRAFT_REPO_ROOT
RUN=${1:-close}
bash scripts/gpu_roundclose.sh $RUN || exit 1
bash scripts/gpu_close_c5.sh ${RUN}_c5 || exit 1
echo all closed
