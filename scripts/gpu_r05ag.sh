#!/bin/bash
# bf16-operand projections: the C5 bench-path parity test alone (diagnostics on refusal)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05ag}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_c5_bench.py > $O/pytest.log 2>&1
echo rc $?
