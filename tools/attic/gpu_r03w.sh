set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
# r03w: the re-created container's rebuild of the round's final source
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/r03w_pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/r03w_bench_c2.json 2> $O/r03w_bench_c2.err &&
timeout -k 10 300 python -u tools/iterbench.py --reps 3 > $O/r03w_iter16.txt 2>&1 &&
timeout -k 10 300 python -u tools/checkcost.py > $O/r03w_checkcost.txt 2>&1
