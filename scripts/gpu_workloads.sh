# Secondary BASELINE workloads on the box: C2 at "high" / "medium", C4 / C5 bench lines at every
# matmul precision, a rocprofv3 kernel summary of each C5 run and the C3 step anatomy.
# usage: bash scripts/gpu_workloads.sh <run-name>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
RUN=${1:-w}
O=gpurun_out/$RUN
mkdir -p $O
for cfg in "c2 high 50 10" "c2 medium 50 10" "c4 highest 30 5" "c4 high 30 5" "c4 medium 30 5" "c5 highest 8 2" "c5 high 10 3" "c5 medium 10 3"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --workload $1 --precision $2 --steps $3 --warmup $4 --skip-cpu \
    > $O/${1}_${2}.json 2> $O/${1}_${2}.err || exit 1
  python3 -c "import json;d=json.load(open('$O/${1}_${2}.json'));print('$1 $2', d['ms_per_step'], d['value'])"
done
for pr in highest high medium; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5_$pr -o run -- \
    python3 bench.py --workload c5 --precision $pr --steps 4 --warmup 1 --skip-cpu --profile-steps 2 \
    > $O/prof_c5_$pr.json 2> $O/prof_c5_$pr.err || exit 1
done
timeout -k 10 600 python -u scripts/c3_encoder_split.py --steps 10 > $O/c3_split.json 2> $O/c3_split.err || exit 1
echo done
