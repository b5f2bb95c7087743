set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/tprof
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_tp.log 2>&1 || { tail -30 gpurun_out/pytest_tp.log; exit 1; }
mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/new -o run -- python3 bench.py --steps 20 --warmup 5 --skip-cpu > $O/new.json 2> $O/new.err || exit 1
MMF_TAIL_GEMV=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/old -o run -- python3 bench.py --steps 20 --warmup 5 --skip-cpu > $O/old.json 2> $O/old.err || exit 1
echo ok
