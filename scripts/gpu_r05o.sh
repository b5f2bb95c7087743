#!/bin/bash
# One-barrier long-key attention forward (C5 "medium"): every GPU test, then the C5 line A/B
# (vs MMF_FWD_TWOBAR=1) and rocprofv3 stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05o}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed rc=$rc"; exit $rc; fi
grep -q "illegal memory access\|Memory access fault" $O/pytest_gpu.log && { echo "GPU fault: stopping"; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu > $O/c5_a$i.json 2> $O/c5_a$i.err || exit $?
  MMF_FWD_TWOBAR=1 timeout -k 10 300 python bench.py --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu > $O/c5_b$i.json 2> $O/c5_b$i.err || exit $?
done
bash scripts/gpu_prof.sh $O c5_medium --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu || exit $?
echo done
