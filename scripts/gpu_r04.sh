#!/bin/bash
# Round-4 evidence in one GPU call: GPU parity tests, smoke, the C2 and C2-L1 bench lines with
# rocprofv3 stats, then the drop-in module / compiled paths.  usage: bash scripts/gpu_r04.sh <run>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r04}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed rc=$rc"; exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
bash scripts/gpu_prof.sh $O c2 --steps 50 --warmup 10 || exit $?
bash scripts/gpu_prof.sh $O c2_l1 --workload c2_l1 --steps 50 --warmup 10 || exit $?
[ -n "${NO_PATHS:-}" ] || bash scripts/gpu_paths.sh $O c2 || exit $?
echo done
