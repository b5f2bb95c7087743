# Bench-only A/B on the box (no tests): one bench line per environment setting.
# usage: bash scripts/gpu_benchab.sh <run-name> "<ENV=VAL ...> [-- <bench args>]" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
RUN=${1:-ab}; shift
O=gpurun_out/$RUN
mkdir -p $O
i=0
for E in "$@"; do
  i=$((i+1))
  EV=${E%% -- *}; BA=""; [ "$EV" != "$E" ] && BA=${E#* -- }
  env $EV timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --skip-cpu --no-graph $BA > $O/bench_$i.json 2> $O/bench_$i.err || exit 1
  python3 -c "import json;d=json.load(open('$O/bench_$i.json'));print('$E', d['ms_per_step'], d['value']);[print('  ',k,v['avg_launch_ms'],v['frac']) for k,v in list(d['kernels'].items())[:6]];print('  ',d['stage_ms'])"
done
