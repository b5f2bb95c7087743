#!/bin/bash
# The L1-path tests, the module-path host profile, the C2-L1 module-path lines, the L1 grid A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05d}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_train_step.py tests/test_gpu_single_key.py tests/test_gpu_headline.py tests/test_gpu_compile.py tests/test_gpu_parity.py -q --timeout 150 --timeout-method thread > $O/pytest_sel.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_sel.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed rc=$rc"; exit $rc; fi
grep -q "illegal memory access\|Memory access fault" $O/pytest_sel.log && { echo "GPU fault: stopping"; exit 1; }
TORCH_LOGS=perf_hints timeout -k 10 400 python -u scripts/host_phase_profile.py --out $O/host_l1.json > $O/host_l1.log 2>&1 || exit $?
bash scripts/gpu_prof.sh $O c2_l1_module --workload c2_l1 --path module --steps 200 --warmup 20 --skip-cpu || exit $?
bash scripts/gpu_prof.sh $O c2_l1_compiled --workload c2_l1 --path compiled --steps 200 --warmup 20 --skip-cpu || exit $?
bash scripts/gpu_l1xcd_ab.sh ${1:-r05d}/xcd || exit $?
echo done
