#!/bin/bash
# PMC passes (one rocprofv3 run per counter group; only --kernel-trace beside --pmc)
# over an eager bench step, so every kernel launch carries its own counters.
# usage: bash profiles/collect_pmc.sh <outdir> [extra bench.py args, e.g. --workload c5 --precision medium]
set -u
OUT=${1:-gpurun_out/pmc}
shift || true
export TMPDIR=/tmp
mkdir -p "$OUT"
B="python3 bench.py --steps 2 --warmup 1 --skip-cpu --no-graph --profile-steps 1 $*"
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- $B \
    > "$OUT/$name.log" 2>&1
}
pass p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
        SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE &&
pass p2 SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_SALU \
        SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_VMEM &&
pass p3 SQ_INSTS_VALU_TRANS_F32 SQ_LEVEL_WAVES SQ_IFETCH SQ_INSTS_SMEM SQ_INST_LEVEL_VMEM \
        SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR
rc=$?
echo "pmc rc=$rc"
[ $rc -eq 0 ] && python3 profiles/pmc_summary.py "$OUT" "$OUT/pmc_summary.json"
