#!/bin/bash
# One bench line + its rocprofv3 kernel-trace summary (only the stats csv is kept: gpurun copies
# back at most 64 MiB).  usage: scripts/gpu_prof.sh <outdir> <tag> [bench args...]
set -o pipefail
OUT=${1:?outdir}; TAG=${2:?tag}; shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python bench.py "$@" > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "/tmp/prof_$TAG" -o run -- python bench.py "$@" --skip-cpu \
    > "$OUT/prof_$TAG.log" 2>&1 || exit $?
f=$(find "/tmp/prof_$TAG" -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cp "$f" "$OUT/${TAG}_kernel_stats.csv"
rm -rf "/tmp/prof_$TAG"
exit 0
