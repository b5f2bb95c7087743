# Same-box A/B of two builds of the library (MMF_LIB_PATH): C2 bench lines alternating
# prev / current.  usage: bash scripts/gpu_ab_lib.sh <run-name> <prev .so (in-tree path)>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
RUN=${1:-ablib}
PREV=${2:-multimodal-sensor-fusion-with-attention-rajeevatla_amd/csrc/libmmfusion_prev.so}
O=gpurun_out/$RUN
mkdir -p $O
for i in 1 2; do
  for v in prev cur; do
    if [ $v = prev ]; then export MMF_LIB_PATH=$GRAFT_REPO_ROOT/$PREV; else unset MMF_LIB_PATH; fi
    timeout -k 10 300 python -u bench.py --workload c2 --steps 50 --warmup 10 --skip-cpu > $O/c2_${v}_$i.json 2> $O/c2_${v}_$i.err || exit 1
    echo "c2 $v $i ok"
  done
done
echo done
