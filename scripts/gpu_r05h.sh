#!/bin/bash
# Every GPU test, then the C2-L1 module / compiled lines with rocprofv3 stats and the host phases.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05h}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed rc=$rc"; exit $rc; fi
grep -q "illegal memory access\|Memory access fault" $O/pytest_gpu.log && { echo "GPU fault in pytest: stopping"; exit 1; }
timeout -k 10 300 python -u scripts/host_phase_profile.py --paths module,compiled --out $O/host_l1.json > $O/host_l1.log 2>&1 || exit $?
bash scripts/gpu_prof.sh $O c2_l1_module --workload c2_l1 --path module --steps 300 --warmup 30 --skip-cpu || exit $?
bash scripts/gpu_prof.sh $O c2_l1_compiled --workload c2_l1 --path compiled --steps 300 --warmup 30 --skip-cpu || exit $?
echo done
