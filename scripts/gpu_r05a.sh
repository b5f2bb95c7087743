#!/bin/bash
# Round-5 first GPU call: the sync-protocol / cross-entropy tests, then the module-path host profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05a}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed rc=$rc"; exit $rc; fi
TORCH_LOGS=perf_hints timeout -k 10 400 python -u scripts/host_phase_profile.py --out $O/host_l1.json > $O/host_l1.log 2>&1 || exit $?
echo done
