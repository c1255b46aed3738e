set -o pipefail
cd $GRAFT_REPO_ROOT
# r05au: part 2 of the round-5 final measurements (gpu_r05at.sh): GPU suite, per-iteration
# latency of C2's / C3's slowest instance and at N = 48 / 64
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/r05au_pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u tools/iterbench.py --N 16 --reps 3 --batches 256 512 > $O/r05au_iter16.txt 2>&1 &&
timeout -k 10 300 python -u tools/iterbench.py --N 32 --reps 3 --batches 256 > $O/r05au_iter32.txt 2>&1 &&
timeout -k 10 300 python -u tools/iterbench.py --N 48 --reps 2 --batches 32 256 > $O/r05au_iter48.txt 2>&1 &&
timeout -k 10 400 python -u tools/iterbench.py --N 64 --reps 2 --batches 32 256 > $O/r05au_iter64.txt 2>&1
