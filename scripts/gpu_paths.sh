#!/bin/bash
# The drop-in module paths of bench.py (eager nn.Module, torch.compile reduce-overhead) beside
# the fused step, each with a rocprofv3 kernel-trace summary.  usage: scripts/gpu_paths.sh <outdir> [workload]
set -o pipefail
OUT=${1:?outdir}; WL=${2:-c2}
for P in step module compiled; do
  bash scripts/gpu_prof.sh "$OUT" "${WL}_${P}" --workload "$WL" --path "$P" --steps 30 --warmup 10 --skip-cpu || exit $?
done
