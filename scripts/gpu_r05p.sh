#!/bin/bash
# GPU timelines of the captured steps (C2, C2-L1, C5 medium): busy vs span per step, the gap before
# each kernel (rocprofv3 kernel trace of the graph replays).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05p}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/kt2 -o run -- python3 bench.py --steps 100 --warmup 20 --skip-cpu > $O/kt_c2.json 2> $O/kt_c2.err || exit $?
f=$(find /tmp/kt2 -name "*kernel_trace.csv" | head -1); cp "$f" $O/kernel_trace_c2.csv
python3 scripts/kernel_timeline.py $O/kernel_trace_c2.csv --first mask_dropout_rows --out $O/timeline_c2.json > /dev/null || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/kt3 -o run -- python3 bench.py --workload c2_l1 --steps 200 --warmup 20 --skip-cpu > $O/kt_l1.json 2> $O/kt_l1.err || exit $?
f=$(find /tmp/kt3 -name "*kernel_trace.csv" | head -1); cp "$f" $O/kernel_trace_l1.csv
python3 scripts/kernel_timeline.py $O/kernel_trace_l1.csv --first l1_fwd_loss --out $O/timeline_l1.json > /dev/null || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/kt5 -o run -- python3 bench.py --workload c5 --precision medium --steps 10 --warmup 3 --skip-cpu > $O/kt_c5.json 2> $O/kt_c5.err || exit $?
f=$(find /tmp/kt5 -name "*kernel_trace.csv" | head -1); cp "$f" $O/kernel_trace_c5.csv
python3 scripts/kernel_timeline.py $O/kernel_trace_c5.csv --first mask_dropout_rows --skip 3 --out $O/timeline_c5.json > /dev/null || exit $?
echo done
