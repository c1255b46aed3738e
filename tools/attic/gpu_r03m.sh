set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
# r03m: beyond 32 stages, the F row in the workspace, the z-update constants batch-loaded, the split sweep's lane ids laundered
timeout -k 10 300 python -u tools/iterbench.py --N 48 --reps 2 > $O/r03m_iter48.txt 2>&1 &&
timeout -k 10 300 python -u tools/iterbench.py --N 64 --reps 2 > $O/r03m_iter64.txt 2>&1 &&
timeout -k 10 300 python -u tools/iterbench.py --N 36 --reps 2 > $O/r03m_iter36.txt 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/r03m_pytest_gpu.log 2>&1
