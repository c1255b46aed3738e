set -o pipefail
cd $GRAFT_REPO_ROOT
# r04v: the LDS exit status up to 16 stages only -- GPU suite, smoke, C2 / C3 lines, C2 rocprof
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04v_pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04v_smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r04v_bench_c2.json 2> gpurun_out/r04v_bench_c2.err &&
timeout -k 10 300 python -u bench.py --config c3 > gpurun_out/r04v_bench_c3.json 2> gpurun_out/r04v_bench_c3.err &&
bash tools/profile.sh r04v --config c2
