# Final round-3 evidence: smoke(), then scripts/gpu_close_r03b.sh (GPU tests, C2 line with CPU legs,
# stats / traffic / SQ, C2 L = 1, C5 medium).  usage: bash scripts/gpu_close_final.sh <run>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/$1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$1/smoke.log 2>&1 || { cat gpurun_out/$1/smoke.log; exit 1; }
tail -1 gpurun_out/$1/smoke.log
bash scripts/gpu_close_r03b.sh $1
