set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_horizons.py -x -v --timeout 300 --timeout-method thread > $O/r03b_horizons.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/r03b_pytest_gpu.log 2>&1 &&
MPCQ_LIB_VARIANT=exp:nozero timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/r03b_nozero.log 2>&1 &&
timeout -k 10 300 python -u tools/iterbench.py --N 48 --reps 3 > $O/r03b_iter48.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:nohold timeout -k 10 300 python -u tools/iterbench.py --N 48 --reps 3 > $O/r03b_iter48_nohold.txt 2>&1 &&
timeout -k 10 300 python -u tools/iterbench.py --N 16 --reps 3 > $O/r03b_iter16.txt 2>&1
