set -o pipefail
cd $GRAFT_REPO_ROOT
# the GPU suite and smoke on the committed final tree (in-tree build from __graft_entry__.build())
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r03end_pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03end_smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r03end_bench_c2.json 2> gpurun_out/r03end_bench_c2.err
