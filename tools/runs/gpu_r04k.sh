set -o pipefail
cd $GRAFT_REPO_ROOT
# r04k: half-wave planner with fsteps straight to HBM, xref read late, 8 waves per SIMD
# (A/B: plnowpe = the same without the occupancy attribute; MPCQ_PLAN_LANES=64 = one robot per wave)
timeout -k 10 600 python -u -m pytest tests/test_gpu_planner.py tests/test_gpu_session.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04k_pytest_planner.log 2>&1 &&
timeout -k 10 300 python -u bench.py --mode plan --cpu-sample 0 > gpurun_out/r04k_bench_plan.json 2> gpurun_out/r04k_bench_plan.err &&
MPCQ_LIB_VARIANT=exp:plnowpe timeout -k 10 300 python -u bench.py --mode plan --cpu-sample 0 > gpurun_out/r04k_bench_plan_nowpe.json 2> gpurun_out/r04k_bench_plan_nowpe.err &&
MPCQ_PLAN_LANES=64 timeout -k 10 300 python -u bench.py --mode plan --cpu-sample 0 > gpurun_out/r04k_bench_plan_l64.json 2> gpurun_out/r04k_bench_plan_l64.err &&
timeout -k 10 300 python -u bench.py --mode plan --cpu-sample 0 > gpurun_out/r04k_bench_plan_2.json 2> gpurun_out/r04k_bench_plan_2.err
