# Diagnostic: C5 long-key kernel times with and without repeat chunk loads (wrong results; timing only)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/c5skip
mkdir -p $O
for P in medium highest; do
  timeout -k 10 200 python -u bench.py --workload c5 --precision $P --steps 10 --warmup 3 --skip-cpu --profile-steps 2 > $O/base_$P.json 2> $O/base_$P.err || exit 1
  MMF_LIB_PATH=scripts/micro/v_skip/libmmfusion.so timeout -k 10 200 python -u bench.py --workload c5 --precision $P --steps 10 --warmup 3 --skip-cpu --profile-steps 2 > $O/skip_$P.json 2> $O/skip_$P.err || exit 1
done
echo ok
