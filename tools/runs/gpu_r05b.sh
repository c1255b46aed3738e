set -o pipefail
cd $GRAFT_REPO_ROOT
# r05b: first run of the explicit-inverse kernel (kKI, N = 16): MFMA f64 layout check, smoke,
# the GPU suite, C2 / C4 / C5 lines, per-iteration latency of C2's slowest instance
O=gpurun_out
timeout -k 10 60 ./tools/ubench/mfl > $O/r05b_mfma_layout.txt 2>&1 &&
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/r05b_smoke.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/r05b_pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/r05b_bench_c2.json 2> $O/r05b_bench_c2.err &&
timeout -k 10 300 python -u tools/iterbench.py --N 16 --reps 3 > $O/r05b_iter16.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:kinv1 timeout -k 10 300 python -u tools/iterbench.py --N 16 --reps 3 > $O/r05b_iter16_norsum.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --config c4 --steps 3 --warmup 1 --restatement 256 --certify 256 > $O/r05b_bench_c4_1gpu.json 2> $O/r05b_bench_c4.err &&
timeout -k 10 300 python -u bench.py --config c5 --steps 3 --warmup 1 --restatement 256 --certify 256 > $O/r05b_bench_c5_1gpu.json 2> $O/r05b_bench_c5.err
