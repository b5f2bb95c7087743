# Round-close evidence in one GPU call: parity tests, PMC traffic passes, the bench line
# (with the CPU baseline), rocprofv3 kernel stats, then the SQ counter passes.
# usage (on the box): bash scripts/gpu_roundclose.sh <run-name>
set -o pipefail
cd $GRAFT_REPO_ROOT
RUN=${1:-close}
bash scripts/gpu_check.sh $RUN || exit 1
bash profiles/collect_pmc.sh gpurun_out/$RUN/sq || exit 1
echo closed
