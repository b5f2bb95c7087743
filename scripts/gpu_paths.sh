#!/bin/bash
# The drop-in module paths of bench.py (eager nn.Module, torch.compile reduce-overhead) beside
# the fused step, each with a rocprofv3 kernel-trace summary.  usage: scripts/gpu_paths.sh <outdir> [workload]
set -o pipefail
OUT=${1:?outdir}; WL=${2:-c2}
mkdir -p "$OUT"
export TMPDIR=/tmp
for P in step module compiled; do
  timeout -k 10 300 python bench.py --workload "$WL" --path "$P" --steps 30 --warmup 10 --skip-cpu \
      > "$OUT/bench_${WL}_${P}.json" 2> "$OUT/bench_${WL}_${P}.err" || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_${WL}_${P}" -o run -- \
      python bench.py --workload "$WL" --path "$P" --steps 30 --warmup 10 --skip-cpu \
      > "$OUT/prof_${WL}_${P}.log" 2>&1 || exit $?
done
