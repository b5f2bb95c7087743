#!/bin/bash
# bench.py without per-step events in the timed region: C2 (with rocprofv3 stats), C2-L1 captured
# vs eager launches.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05r}
mkdir -p $O
bash scripts/gpu_prof.sh $O c2 --steps 200 --warmup 20 || exit $?
for i in 1 2; do
  timeout -k 10 200 python bench.py --workload c2_l1 --steps 500 --warmup 50 --skip-cpu > $O/l1_graph$i.json 2> $O/l1_graph$i.err || exit $?
  timeout -k 10 200 python bench.py --workload c2_l1 --steps 500 --warmup 50 --skip-cpu --no-graph > $O/l1_eager$i.json 2> $O/l1_eager$i.err || exit $?
done
echo done
