set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
# r03t: the final build: GPU suite, smoke, C2 bench line
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/r03t_pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r03t_smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/r03t_bench_c2.json 2> $O/r03t_bench_c2.err
