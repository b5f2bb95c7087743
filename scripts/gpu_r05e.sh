#!/bin/bash
# Round-5 measurement call: the module path's native / Python host split, the C2-L1 fused-step line
# with rocprofv3 stats, the SQ counter passes for C2-L1, C5 "medium" and C2, and the C5 line with its
# CPU leg.  usage (on the box): bash scripts/gpu_r05e.sh <run-name>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05e}
mkdir -p $O
timeout -k 10 300 python -u scripts/host_native_probe.py --out $O/native_probe.json > $O/native_probe.log 2>&1 || exit $?
bash scripts/gpu_prof.sh $O c2_l1_step --workload c2_l1 --path step --steps 300 --warmup 30 --skip-cpu || exit $?
timeout -k 10 300 bash profiles/collect_pmc.sh $O/pmc_c2_l1 --workload c2_l1 > $O/pmc_c2_l1.log 2>&1 || exit $?
timeout -k 10 400 bash profiles/collect_pmc.sh $O/pmc_c5 --workload c5 --precision medium > $O/pmc_c5.log 2>&1 || exit $?
timeout -k 10 500 python bench.py --workload c5 --precision medium --steps 20 --warmup 5 > $O/bench_c5_medium.json 2> $O/bench_c5_medium.err || exit $?
timeout -k 10 300 bash profiles/collect_pmc.sh $O/pmc_c2 > $O/pmc_c2.log 2>&1 || exit $?
echo done
