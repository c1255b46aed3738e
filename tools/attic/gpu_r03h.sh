set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python -u tools/iterbench.py --N 16 --reps 3 > $O/r03h_iter16.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/r03h_pytest_gpu.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc   # test failures go on to the timings; a crash or time limit stops here
MPCQ_LIB_VARIANT=exp:lagging timeout -k 10 300 python -u tools/iterbench.py --N 16 --reps 3 > $O/r03h_iter16_lagging.txt 2>&1 &&
timeout -k 10 300 python -u tools/iterbench.py --N 32 --reps 3 > $O/r03h_iter32.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:lagging timeout -k 10 300 python -u tools/iterbench.py --N 32 --reps 3 > $O/r03h_iter32_lagging.txt 2>&1 &&
timeout -k 10 300 python -u tools/iterbench.py --N 48 --reps 2 > $O/r03h_iter48.txt 2>&1
