set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-diag}
mkdir -p $O
DIAG_P=0 timeout -k 10 300 python -u scripts/diag_train_case.py train_pipe highest > $O/highest_p0.txt 2>&1 || exit 1
DIAG_P=0 MMF_FWD_PIPE=0 timeout -k 10 300 python -u scripts/diag_train_case.py train_pipe highest > $O/highest_p0_nopipe.txt 2>&1 || exit 1
DIAG_P=0 MMF_FWD_PIPE=0 timeout -k 10 300 python -u scripts/diag_train_case.py train_pipe high > $O/high_p0_nopipe.txt 2>&1 || exit 1
DIAG_P=0 MMF_NO_WSR=1 timeout -k 10 300 python -u scripts/diag_train_case.py train_pipe high > $O/high_p0_nowsr.txt 2>&1 || exit 1
echo done
