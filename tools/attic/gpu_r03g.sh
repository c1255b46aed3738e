set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
bash tools/gpu_mp_rehearsal.sh r03g &&
timeout -k 10 300 python -u bench.py --mode plan --cpu-sample 4096 > $O/r03g_bench_plan.json 2> $O/r03g_bench_plan.err &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_horizons.py tests/test_gpu_parity.py tests/test_gpu_session.py -x -v -rP --timeout 300 --timeout-method thread > $O/r03g_prints.log 2>&1
