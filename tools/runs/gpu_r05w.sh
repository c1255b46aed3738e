set -o pipefail
cd $GRAFT_REPO_ROOT
# r05w: round-5 final build (instruction cuts, exit status carried beyond 48 stages): smoke, every bench line of
# DESIGN §5, the stamped rocprof passes for C2 and C3, GPU suite, per-iteration at N = 16..64
O=gpurun_out
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/r05w_smoke.log 2>&1 &&
bash tools/bench_all.sh r05w &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/r05w_pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u tools/iterbench.py --N 16 --reps 3 --batches 256 512 > $O/r05w_iter16.txt 2>&1 &&
timeout -k 10 300 python -u tools/iterbench.py --N 32 --reps 3 --batches 256 > $O/r05w_iter32.txt 2>&1 &&
timeout -k 10 300 python -u tools/iterbench.py --N 48 --reps 2 --batches 32 256 > $O/r05w_iter48.txt 2>&1 &&
timeout -k 10 400 python -u tools/iterbench.py --N 64 --reps 2 --batches 32 256 > $O/r05w_iter64.txt 2>&1
