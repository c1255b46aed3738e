set -o pipefail
cd $GRAFT_REPO_ROOT
# r04u: the ADMM exit status through LDS (no loop-carried status register) -- GPU suite, smoke,
# same-box A/B of the per-iteration latency (prev = before, cur = this), C2 / C3 lines + rocprof
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04u_pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04u_smoke.log 2>&1 &&
for v in prev16 cur16 prev16 cur16; do
  MPCQ_LIB_VARIANT=exp:$v timeout -k 10 180 python -u tools/iterbench.py --N 16 --reps 3 --batches 256 512 >> gpurun_out/r04u_ab16.txt 2>&1 || exit 1
done &&
for v in prev32 cur32 prev32 cur32; do
  MPCQ_LIB_VARIANT=exp:$v timeout -k 10 180 python -u tools/iterbench.py --N 32 --reps 3 --batches 256 >> gpurun_out/r04u_ab32.txt 2>&1 || exit 1
done &&
timeout -k 10 300 python -u bench.py > gpurun_out/r04u_bench_c2.json 2> gpurun_out/r04u_bench_c2.err &&
timeout -k 10 300 python -u bench.py --config c3 > gpurun_out/r04u_bench_c3.json 2> gpurun_out/r04u_bench_c3.err &&
bash tools/profile.sh r04u --config c2 &&
bash tools/profile.sh r04uc3 --config c3
