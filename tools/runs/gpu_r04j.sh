set -o pipefail
cd $GRAFT_REPO_ROOT
# r04j: the planner with two instances per wave64 (N <= 31) -- planner + session GPU tests,
# plan / tick bench lines, same-box A/B against one instance per wave (MPCQ_PLAN_LANES=64)
timeout -k 10 600 python -u -m pytest tests/test_gpu_planner.py tests/test_gpu_session.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04j_pytest_planner.log 2>&1 &&
timeout -k 10 300 python -u bench.py --mode plan --cpu-sample 0 > gpurun_out/r04j_bench_plan.json 2> gpurun_out/r04j_bench_plan.err &&
MPCQ_PLAN_LANES=64 timeout -k 10 300 python -u bench.py --mode plan --cpu-sample 0 > gpurun_out/r04j_bench_plan_l64.json 2> gpurun_out/r04j_bench_plan_l64.err &&
timeout -k 10 300 python -u bench.py --mode plan --cpu-sample 0 > gpurun_out/r04j_bench_plan_2.json 2> gpurun_out/r04j_bench_plan_2.err &&
timeout -k 10 300 python -u bench.py --mode tick --steps 20 --warmup 4 --cpu-sample 0 > gpurun_out/r04j_bench_tick_c2.json 2> gpurun_out/r04j_bench_tick_c2.err
