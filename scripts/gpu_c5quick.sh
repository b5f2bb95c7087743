# Quick C5 loop: long-key parity tests, then C5 bench at every precision (top kernels).
set -o pipefail
cd $GRAFT_REPO_ROOT
RUN=${1:-c5q}
O=gpurun_out/$RUN
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_train_mode.py tests/test_gpu_bf16.py -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "^E  |passed|failed|Error" $O/pytest_gpu.log | head -20
[ $rc -ne 0 ] && exit $rc
for pr in highest high medium; do
  timeout -k 10 300 python -u bench.py --workload c5 --precision $pr --steps 6 --warmup 2 --skip-cpu > $O/c5_$pr.json 2> $O/c5_$pr.err || exit 1
  python3 -c "import json;d=json.load(open('$O/c5_$pr.json'));print('$pr', d['ms_per_step'], d['value']);[print('  ',k,v['ms_per_step']) for k,v in list(d['kernels'].items())[:5]]"
done
