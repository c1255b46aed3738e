set -o pipefail
cd $GRAFT_REPO_ROOT
# r04g: the workspace (N > 32) read through global-address-space pointers -- GPU suite,
# per-iteration latency and stamps beyond 32 stages
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04g_pytest_gpu.log 2>&1 &&
for n in 40 48 49 56 64; do
  timeout -k 10 180 python -u tools/iterbench.py --N $n --reps 2 --batches 32 256 > gpurun_out/r04g_iter$n.txt 2>&1 || exit 1
done &&
for n in 48 64; do
  timeout -k 10 120 python -u tools/stamps.py --N $n --batch 256 > gpurun_out/r04g_stamps$n.txt 2>&1 || exit 1
done
