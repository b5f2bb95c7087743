#!/bin/bash
# Graph-replay boundary: per-step event records vs none (C2-L1, C2); the split pool_u on C5.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05q}
mkdir -p $O
timeout -k 10 300 python -u scripts/replay_gap_probe.py --workload c2_l1 --steps 1000 > $O/gap_l1.json 2> $O/gap_l1.err || exit $?
timeout -k 10 300 python -u scripts/replay_gap_probe.py --workload c2 --steps 200 > $O/gap_c2.json 2> $O/gap_c2.err || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_c5_bench.py tests/test_gpu_bf16.py tests/test_gpu_train_mode.py tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed rc=$rc"; exit $rc; fi
grep -q "illegal memory access\|Memory access fault" $O/pytest.log && { echo "GPU fault: stopping"; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu > $O/c5_a$i.json 2> $O/c5_a$i.err || exit $?
  MMF_POOLU_NOSPLIT=1 timeout -k 10 300 python bench.py --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu > $O/c5_b$i.json 2> $O/c5_b$i.err || exit $?
done
echo done
