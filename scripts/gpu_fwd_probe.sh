# Forward attention probe: the C2 bench with and without dropout (the lean forward's
# Philox keep-bit draws run inside its load window) + the stamp breakdown without dropout.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-fwdp}
mkdir -p $O
timeout -k 10 300 python -u bench.py --skip-cpu --dropout 0 > $O/bench_p0.json 2> $O/bench_p0.err || exit 1
timeout -k 10 300 python -u bench.py --skip-cpu > $O/bench_p01.json 2> $O/bench_p01.err || exit 1
echo done
