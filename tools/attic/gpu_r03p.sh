set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
# r03p: F row / z constants in memory beyond 48 stages only
timeout -k 10 300 python -u tools/bigsweep.py > $O/r03p_sweep.txt 2>&1 &&
timeout -k 10 300 python -u tools/iterbench.py --N 48 --reps 2 > $O/r03p_iter48.txt 2>&1 &&
timeout -k 10 300 python -u tools/iterbench.py --N 64 --reps 2 > $O/r03p_iter64.txt 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/r03p_pytest_gpu.log 2>&1
