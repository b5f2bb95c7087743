# One bench workload under several environment settings, same box (top kernels).
# usage (on the box): bash scripts/gpu_env_ab.sh <run-name> "<bench args>" "<ENV=VAL ...>" ["<ENV=VAL ...>" ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
RUN=${1:-envab}; shift
ARGS=$1; shift
O=gpurun_out/$RUN
mkdir -p $O
i=0
for E in "$@"; do
  i=$((i+1))
  env $E timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --skip-cpu $ARGS > $O/bench_$i.json 2> $O/bench_$i.err || exit 1
  python3 -c "import json;d=json.load(open('$O/bench_$i.json'));print('$E', d['ms_per_step'], d['value']);[print('   %-40s %8.1f us' % (k[:40], v['avg_launch_ms']*1e3)) for k,v in list(d['kernels'].items())[:12] if 'tail' in k]"
done
