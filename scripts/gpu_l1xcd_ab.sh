#!/bin/bash
# L = 1 grid layout A/B: the L1 GPU tests on the product library (plain (tile, pair) ids), then the
# C2-L1 line alternating the product library (A) and libmmfusion_l1xcd.so (B: XCD-major ids, `make
# l1xcd`), and the FETCH_SIZE / WRITE_SIZE passes of both.  usage: bash scripts/gpu_l1xcd_ab.sh <run>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-l1xcd}
mkdir -p $O
P=multimodal-sensor-fusion-with-attention-rajeevatla_amd/csrc
timeout -k 10 300 python -u -m pytest tests/test_gpu_train_step.py tests/test_gpu_single_key.py tests/test_gpu_headline.py -x -q --timeout 120 --timeout-method thread > $O/pytest_l1.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 120 python bench.py --workload c2_l1 --steps 300 --warmup 30 --skip-cpu > $O/a$i.json 2> $O/a$i.err || exit $?
  timeout -k 10 120 env MMF_LIB_PATH=$P/libmmfusion_l1xcd.so python bench.py --workload c2_l1 --steps 300 --warmup 30 --skip-cpu > $O/b$i.json 2> $O/b$i.err || exit $?
done
PB="python3 bench.py --workload c2_l1 --steps 2 --warmup 1 --skip-cpu --no-graph --profile-steps 1"
for V in a b; do
  [ $V = b ] && export MMF_LIB_PATH=$P/libmmfusion_l1xcd.so
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d /tmp/pf_$V -o run -- $PB > $O/pmc_fetch_$V.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d /tmp/pw_$V -o run -- $PB > $O/pmc_write_$V.log 2>&1 || exit 1
  python3 profiles/pmc_traffic.py /tmp/pf_$V/run_counter_collection.csv /tmp/pw_$V/run_counter_collection.csv "l1 xcd A/B ($V): $PB" $O/pmc_traffic_$V.json || exit 1
  unset MMF_LIB_PATH
done
echo done
