#!/bin/bash
# L1 A/B: the L1 GPU tests on the product library, then the C2-L1 line alternating the product
# library (A) and libmmfusion_exp.so (B), and the stamps of both.  B is built beforehand from the
# product objects with l1.hip recompiled under the variant's -D flag (and libmmfusion_expst.so with
# -DMMF_STAMPS added), e.g. in csrc/: hipcc $(CXXFLAGS) -DVARIANT -c l1.hip -o /tmp/l1.o &&
# hipcc -shared --offload-arch=gfx950 -o libmmfusion_exp.so <the other .o files> /tmp/l1.o
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-l1ab}
mkdir -p $O
P=multimodal-sensor-fusion-with-attention-rajeevatla_amd/csrc
timeout -k 10 300 python -u -m pytest tests/test_gpu_train_step.py tests/test_gpu_single_key.py tests/test_gpu_headline.py -x -q --timeout 120 --timeout-method thread > $O/pytest_l1.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 120 python bench.py --workload c2_l1 --steps 200 --warmup 20 --skip-cpu > $O/a$i.json 2> $O/a$i.err || exit $?
  timeout -k 10 120 env MMF_LIB_PATH=$P/libmmfusion_exp.so python bench.py --workload c2_l1 --steps 200 --warmup 20 --skip-cpu > $O/b$i.json 2> $O/b$i.err || exit $?
done
timeout -k 10 120 env MMF_LIB_PATH=$P/libmmfusion_stampsl1.so python scripts/l1_stamps.py > $O/stamps_a.json 2> $O/stamps_a.err || exit $?
timeout -k 10 120 env MMF_LIB_PATH=$P/libmmfusion_expst.so python scripts/l1_stamps.py > $O/stamps_b.json 2> $O/stamps_b.err || exit $?
echo done
