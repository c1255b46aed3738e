set -o pipefail
cd $GRAFT_REPO_ROOT
# r05i: the production build with lazy Gauss-Jordan pivot rows: GPU suite, smoke
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/r05i_pytest_gpu.log 2>&1 &&
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/r05i_smoke.log 2>&1
