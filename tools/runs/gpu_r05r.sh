set -o pipefail
cd $GRAFT_REPO_ROOT
# r05r: production build with the right-hand-side cuts: GPU suite, smoke, per-iteration at
# N = 16 / 32 / 48 / 64, C2 and C3 lines
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/r05r_pytest_gpu.log 2>&1 &&
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/r05r_smoke.log 2>&1 &&
timeout -k 10 200 python -u tools/iterbench.py --N 16 --reps 3 --batches 256 512 > $O/r05r_iter16.txt 2>&1 &&
timeout -k 10 200 python -u tools/iterbench.py --N 32 --reps 3 --batches 256 > $O/r05r_iter32.txt 2>&1 &&
timeout -k 10 300 python -u tools/iterbench.py --N 48 --reps 2 --batches 32 256 > $O/r05r_iter48.txt 2>&1 &&
timeout -k 10 400 python -u tools/iterbench.py --N 64 --reps 2 --batches 32 256 > $O/r05r_iter64.txt 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/r05r_bench_c2.json 2> $O/r05r_bench_c2.err &&
timeout -k 10 300 python -u bench.py --config c3 > $O/r05r_bench_c3.json 2> $O/r05r_bench_c3.err
