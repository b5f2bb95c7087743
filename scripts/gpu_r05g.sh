#!/bin/bash
# The module path's timelines: the C++-node test, the CPU chrome traces of the module / compiled
# paths, and the GPU kernel timeline (rocprofv3 kernel trace) of the module path.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05g}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_torch_ext.py -v --timeout 150 --timeout-method thread > $O/pytest_ext.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/host_phase_profile.py --paths module,compiled --trace $O/trace --out $O/host_l1.json > $O/host_l1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/kt -o run -- python3 bench.py --workload c2_l1 --path module --steps 200 --warmup 20 --skip-cpu > $O/kt_bench.json 2> $O/kt_bench.err || exit $?
f=$(find /tmp/kt -name "*kernel_trace.csv" | head -1)
cp "$f" $O/kernel_trace_module.csv
python3 scripts/kernel_timeline.py $O/kernel_trace_module.csv --first l1_pair_fwd --out $O/timeline_module.json > /dev/null || exit $?
timeout -k 10 300 python -u scripts/gemm_probe.py --out $O/gemm_probe.json > $O/gemm_probe.log 2>&1 || exit $?
echo done
