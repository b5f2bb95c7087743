#!/bin/bash
# Round-6 GPU call: the new / changed parity tests first, then the whole -m gpu suite, the
# timed-region probe, the driver's exact bench command and its rocprofv3 kernel trace.
# usage (on the box): bash scripts/gpu_r06.sh <run-name> [quick]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
RUN=${1:?run name}
O=gpurun_out/$RUN
mkdir -p "$O"
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $PYT tests/test_gpu_c4_bench.py "tests/test_gpu_train_step.py::test_plan_switch_after_sizing_is_refused" \
    "tests/test_dp.py::test_dp_two_ranks_gpu_matches_single_process" tests/test_gpu_torch_ext.py \
    "tests/test_gpu_train_step.py::test_l1_poll_timeout_surfaces_and_recovers" > "$O/pytest_new.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$O/pytest_new.log"
[ $rc -ne 0 ] && { echo "new tests failed rc=$rc"; tail -40 "$O/pytest_new.log"; exit $rc; }
[ "$2" = "quick" ] && { echo done-quick; exit 0; }
timeout -k 10 900 $PYT tests -m gpu > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$O/pytest_gpu.log"
[ $rc -ne 0 ] && { echo "gpu suite failed rc=$rc"; tail -40 "$O/pytest_gpu.log"; exit $rc; }
timeout -k 10 300 python -u scripts/timed_gap_probe.py --steps 20 --warmup 5 > "$O/gap_probe.json" 2> "$O/gap_probe.err" || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_driver.json" 2> "$O/bench_driver.err" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/ktrace" -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 \
    > "$O/ktrace_bench.json" 2> "$O/ktrace.err" || exit 1
echo done
