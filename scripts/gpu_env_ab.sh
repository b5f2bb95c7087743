# Same-box A/B of the C2 step under plan switches read from the environment:
# default, MMF_SIDE_STREAM=1 (keep words on a side stream), MMF_PSTORE=1 (stored probabilities),
# MMF_KW_SERIAL=1 (keep words drawn on the step's stream ahead of the projection GEMM),
# MMF_KW_FUSED=1 (keep words drawn by extra workgroups of the input-mask kernel, also with long
# keys), MMF_NO_KW_FUSED=1 ("nofused": without them).
# WORKLOAD=c5 PRECISION=medium select another workload.
# usage: bash scripts/gpu_env_ab.sh <run-name> [variant ...]   (default: default side pstore)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-envab}
shift
VARS="${@:-default side pstore}"
mkdir -p $O
for i in 1 2; do
  for v in $VARS; do
    unset MMF_SIDE_STREAM MMF_PSTORE MMF_KW_SERIAL MMF_KW_FUSED MMF_NO_KW_FUSED
    [ $v = nofused ] && export MMF_NO_KW_FUSED=1
    [ $v = fused ] && export MMF_KW_FUSED=1
    [ $v = serial ] && export MMF_KW_SERIAL=1
    [ $v = side ] && export MMF_SIDE_STREAM=1
    [ $v = pstore ] && export MMF_PSTORE=1
    timeout -k 10 300 python -u bench.py --workload ${WORKLOAD:-c2} --precision ${PRECISION:-highest} --steps ${STEPS:-50} --warmup 10 --skip-cpu > $O/${WORKLOAD:-c2}_${v}_$i.json 2> $O/${WORKLOAD:-c2}_${v}_$i.err || exit 1
    echo "$v $i ok"
  done
done
echo done
