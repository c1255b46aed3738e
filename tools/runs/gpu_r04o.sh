set -o pipefail
cd $GRAFT_REPO_ROOT
# r04o: the folded factorisation forms restricted to N <= 32 -- GPU suite, N = 48 / 64 latency
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04o_pytest_gpu.log 2>&1 &&
for n in 48 64; do
  timeout -k 10 180 python -u tools/iterbench.py --N $n --reps 2 --batches 32 256 > gpurun_out/r04o_iter$n.txt 2>&1 || exit 1
done
