set -o pipefail
cd $GRAFT_REPO_ROOT
# r05t: beyond 48 stages the right-hand-side laundering restored: per-iteration at N = 48 / 56
# / 64 and the horizon GPU tests
O=gpurun_out
timeout -k 10 300 python -u tools/iterbench.py --N 48 --reps 2 --batches 32 256 > $O/r05t_iter48.txt 2>&1 &&
timeout -k 10 400 python -u tools/iterbench.py --N 56 --reps 2 --batches 32 256 > $O/r05t_iter56.txt 2>&1 &&
timeout -k 10 400 python -u tools/iterbench.py --N 64 --reps 2 --batches 32 256 > $O/r05t_iter64.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_horizons.py tests/test_gpu_session.py -x -v --timeout 300 --timeout-method thread > $O/r05t_pytest_horizons.log 2>&1
