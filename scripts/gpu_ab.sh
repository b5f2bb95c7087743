#!/bin/bash
# Same-box A/B of bench.py lines under environment settings, alternating the arms R times.
# usage (on the box): bash scripts/gpu_ab.sh <run-name> <R> "<label>:<VAR=v,VAR2=w|->" ... -- [bench args]
#   e.g. bash scripts/gpu_ab.sh r06b 2 "base:-" "ilv2:MMF_GEMM_ILV=2" -- --steps 20 --warmup 5 --skip-cpu
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:?run name}; shift
R=${1:?repeats}; shift
ARMS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do ARMS+=("$1"); shift; done
[ "$1" = "--" ] && shift
mkdir -p "$O"
for i in $(seq 1 "$R"); do
  for arm in "${ARMS[@]}"; do
    label=${arm%%:*}; envs=${arm#*:}
    (
      if [ "$envs" != "-" ]; then
        IFS=',' read -ra kv <<< "$envs"
        for e in "${kv[@]}"; do export "$e"; done
      fi
      timeout -k 10 300 python -u bench.py "$@" > "$O/${label}_$i.json" 2> "$O/${label}_$i.err"
    ) || { echo "arm $label run $i failed"; exit 1; }
    echo "$label $i $(python3 -c "import json,sys;d=json.loads(open('$O/${label}_$i.json').read().strip().splitlines()[-1]);print(d['ms_per_step'],d['ms_per_step_median'])")"
  done
done
echo done
