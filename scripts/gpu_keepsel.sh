# keep_sel in the pooled forward / fused backward: GPU tests, then C2 A/B against the HEAD build.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-keepsel}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log; tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash scripts/gpu_ab_lib.sh $1/ab multimodal-sensor-fusion-with-attention-rajeevatla_amd/csrc/libmmfusion_base.so || exit 1
echo done
