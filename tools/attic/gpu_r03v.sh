set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
# r03v: split sweep's rotation as a select (no exec branch) beyond 32 stages
timeout -k 10 300 python -u tools/bigsweep.py > $O/r03v_sweep.txt 2>&1 &&
timeout -k 10 300 python -u tools/iterbench.py --N 48 --reps 2 > $O/r03v_iter48.txt 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/r03v_pytest_gpu.log 2>&1
