# Same-box A/B of library builds (csrc/libmmfusion_<cfg>.so through MMF_LIB_PATH; "cur" = the
# in-tree build) on C4 at every matmul precision.
# usage: bash scripts/gpu_c4_ab.sh <run-name> <cfg> [<cfg> ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
RUN=$1; shift
O=gpurun_out/$RUN
mkdir -p $O
C=multimodal-sensor-fusion-with-attention-rajeevatla_amd/csrc
for i in 1 2; do
  for v in "$@"; do
    if [ $v = cur ]; then unset MMF_LIB_PATH; else export MMF_LIB_PATH=$GRAFT_REPO_ROOT/$C/libmmfusion_$v.so; fi
    for pr in highest high medium; do
      timeout -k 10 300 python -u bench.py --workload c4 --precision $pr --steps 40 --warmup 10 --skip-cpu > $O/c4_${pr}_${v}_$i.json 2> $O/c4_${pr}_${v}_$i.err || exit 1
    done
    echo "$v $i ok"
  done
done
for v in "$@"; do
  if [ $v = cur ]; then unset MMF_LIB_PATH; else export MMF_LIB_PATH=$GRAFT_REPO_ROOT/$C/libmmfusion_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python3 bench.py --workload c4 --precision medium --steps 10 --warmup 3 --skip-cpu > $O/prof_$v.json 2> $O/prof_$v.err || exit 1
  echo "prof $v ok"
done
echo done
