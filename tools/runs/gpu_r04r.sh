set -o pipefail
cd $GRAFT_REPO_ROOT
# r04r: the widened F W last in LDS (N <= 32), in place beyond -- GPU suite, C2 / C3 lines, rocprof
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04r_pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04r_smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r04r_bench_c2.json 2> gpurun_out/r04r_bench_c2.err &&
timeout -k 10 300 python -u bench.py --config c3 > gpurun_out/r04r_bench_c3.json 2> gpurun_out/r04r_bench_c3.err &&
bash tools/profile.sh r04r --config c2 &&
bash tools/profile.sh r04rc3 --config c3
