set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/r03d_pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u tools/iterbench.py --N 48 --reps 3 > $O/r03d_iter48.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:stamps48 timeout -k 10 300 python -u tools/stamps.py --N 48 --batch 256 --copies 2 > $O/r03d_stamps48.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:stamps48 timeout -k 10 300 python -u tools/stamps.py --N 32 --batch 256 --copies 0 > $O/r03d_stamps32.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --config c2 > $O/r03d_bench_c2.json 2> $O/r03d_bench_c2.err &&
timeout -k 10 300 python -u bench.py --config c3 > $O/r03d_bench_c3.json 2> $O/r03d_bench_c3.err
