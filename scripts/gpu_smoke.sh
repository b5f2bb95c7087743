#!/bin/bash
# __graft_entry__.smoke() on the box (the driver's round-end check), alone
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/${1:-smoke}
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${1:-smoke}/smoke.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/${1:-smoke}/smoke.log; exit $rc
