# A/B of library builds on ONE box: for each in-tree .so, the bench line (graph replay,
# step time) and a rocprofv3 kernel-stats pass (per-kernel average durations).
# usage (on the box): bash scripts/gpu_abprof.sh <run-name> <lib.so> [<lib.so> ...] [-- bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
RUN=${1:-abp}; shift
LIBS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
[ "$1" == "--" ] && shift
O=gpurun_out/$RUN
mkdir -p $O
i=0
for L in "${LIBS[@]}"; do
  i=$((i+1))
  MMF_LIB_PATH=$PWD/$L timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --skip-cpu "$@" > $O/bench_$i.json 2> $O/bench_$i.err || exit 1
  MMF_LIB_PATH=$PWD/$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$i -o run -- python3 bench.py --steps 30 --warmup 5 --skip-cpu "$@" > $O/prof_$i.json 2> $O/prof_$i.err || exit 1
  python3 - "$O" "$i" "$L" <<'EOF'
import csv, glob, json, sys
o, i, lib = sys.argv[1:4]
d = json.load(open(f"{o}/bench_{i}.json"))
print(f"[{i}] {lib}: {d['ms_per_step']} ms/step, {d['value']} samples/s")
f = glob.glob(f"{o}/prof_{i}/**/run_kernel_stats.csv", recursive=True)
rows = list(csv.DictReader(open(f[0])))
tot = 0.0
for r in rows:
    n = r["Name"]
    if "mmf::" not in n:
        continue
    avg = float(r["AverageNs"]) / 1000
    tot += float(r["TotalDurationNs"]) / 1000
    short = n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].split("::")[-1][:60]
    print(f"    {short:60s} {avg:8.1f} us x{r['Calls']}")
print(f"    total mmf kernel time {tot:.0f} us")
EOF
done
