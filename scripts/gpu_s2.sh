# C2 L = 1 and C5 medium lines with the workload-specific PMC traffic lookup; hipBLASLt's kernel
# choices for the C2 GEMM shapes (rocprofv3 kernel names of scripts/lib_gemm_ceiling.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-s2}
mkdir -p $O
timeout -k 10 300 python -u bench.py --workload c2_l1 --skip-cpu > $O/bench_c2_l1.json 2> $O/bench_c2_l1.err || exit 1
timeout -k 10 300 python -u bench.py --workload c5 --precision medium --skip-cpu > $O/bench_c5m.json 2> $O/bench_c5m.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/libprof -o run -- python3 scripts/lib_gemm_ceiling.py > $O/lib_gemm.json 2> $O/lib_gemm.err || exit 1
echo done
