set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
# lane offsets re-derived in the check (every N) and the loop phases (N > 32)
timeout -k 10 300 python -u tools/checkcost.py --N 16 > $O/r03j_check16.txt 2>&1 &&
timeout -k 10 300 python -u tools/iterbench.py --N 16 --reps 3 > $O/r03j_iter16.txt 2>&1 &&
timeout -k 10 300 python -u tools/iterbench.py --N 48 --reps 2 > $O/r03j_iter48.txt 2>&1 &&
timeout -k 10 300 python -u tools/checkcost.py --N 32 > $O/r03j_check32.txt 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/r03j_pytest_gpu.log 2>&1
