#!/bin/bash
# C5: 128 x 256 tiles for the RK x KR bf16 form (dZ and, now on bf16 operands, dX) A/B (MMF_GEMM_WIDE_DZ=1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05am}
mkdir -p $O
# (the C5 parity test asserts the default kernel names: run it without the env var)
B="python bench.py --workload c5 --precision medium --steps 20 --warmup 5 --skip-cpu"
for i in 1 2; do
  timeout -k 10 200 $B > $O/c5_def_$i.json 2> $O/c5_def_$i.err || exit $?
  timeout -k 10 200 env MMF_GEMM_WIDE_DZ=1 $B > $O/c5_wide_$i.json 2> $O/c5_wide_$i.err || exit $?
done
echo done
