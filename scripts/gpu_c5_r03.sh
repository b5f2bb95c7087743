# Round-3 C5 evidence: bench lines at the three precisions, then rocprofv3 kernel stats,
# HBM traffic and SQ passes of the bf16 ("medium") step.  usage: bash scripts/gpu_c5_r03.sh <run-name>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
RUN=${1:-c5r3}
O=gpurun_out/$RUN
mkdir -p $O
for pr in medium high highest; do
  timeout -k 10 300 python -u bench.py --workload c5 --precision $pr --steps 20 --warmup 5 --skip-cpu > $O/c5_${pr}_bench.json 2> $O/c5_${pr}.err || exit 1
  echo "c5 $pr ok"
done
bash scripts/gpu_profile_r03.sh $RUN/c5m --workload c5 --precision medium || exit 1
echo done
