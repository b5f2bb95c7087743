#!/bin/bash
# Final check at the head: full GPU suite, smoke(), the C2 and C5 bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-final}
mkdir -p $O
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --skip-cpu > $O/bench_c2.json 2> $O/bench_c2.err || exit $?
timeout -k 10 300 python -u bench.py --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
echo done
