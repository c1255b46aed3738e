set -o pipefail
cd $GRAFT_REPO_ROOT
# r04q: the round-4 final source (after the F W stride) -- GPU suite, smoke, every bench line, the rocprof passes
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04q_pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04q_smoke.log 2>&1 &&
bash tools/bench_all.sh r04q
