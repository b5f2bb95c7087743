#!/bin/bash
# Round-5 measurement call: the L = 1 module paths (eager, compiled) with rocprofv3 stats, the SQ
# counter passes for C2, C2-L1 and C5 "medium", and the C5 line with its CPU leg.
# usage (on the box): bash scripts/gpu_r05b.sh <run-name>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
RUN=${1:-r05b}
O=gpurun_out/$RUN
mkdir -p $O
for P in module compiled step; do
  bash scripts/gpu_prof.sh $O c2_l1_$P --workload c2_l1 --path $P --steps 100 --warmup 20 --skip-cpu || exit $?
done
timeout -k 10 300 bash profiles/collect_pmc.sh $O/pmc_c2 > $O/pmc_c2.log 2>&1 || exit $?
timeout -k 10 300 bash profiles/collect_pmc.sh $O/pmc_c2_l1 --workload c2_l1 > $O/pmc_c2_l1.log 2>&1 || exit $?
timeout -k 10 400 bash profiles/collect_pmc.sh $O/pmc_c5 --workload c5 --precision medium > $O/pmc_c5.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --workload c5 --precision medium --steps 20 --warmup 5 > $O/bench_c5_medium.json 2> $O/bench_c5_medium.err || exit $?
echo done
