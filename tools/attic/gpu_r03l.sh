set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
# r03l: check constants batch-loaded up to 32 stages, direct beyond
timeout -k 10 300 python -u tools/checkcost.py --N 16 > $O/r03l_check16.txt 2>&1 &&
timeout -k 10 300 python -u tools/checkcost.py --N 32 > $O/r03l_check32.txt 2>&1 &&
timeout -k 10 300 python -u tools/iterbench.py --N 16 --reps 3 > $O/r03l_iter16.txt 2>&1 &&
timeout -k 10 300 python -u tools/iterbench.py --N 32 --reps 2 > $O/r03l_iter32.txt 2>&1 &&
timeout -k 10 300 python -u tools/iterbench.py --N 48 --reps 2 > $O/r03l_iter48.txt 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/r03l_pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/r03l_bench_c2.json 2> $O/r03l_bench_c2.err
