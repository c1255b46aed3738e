set -o pipefail
cd $GRAFT_REPO_ROOT
# r04p: F W at a 96-double stage stride up to 32 stages (ph_recover's row reads without
# bank conflicts) -- GPU suite, per-iteration latency, C2 / C3 lines, the C3 rocprof passes
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04p_pytest_gpu.log 2>&1 &&
for n in 16 32; do
  timeout -k 10 180 python -u tools/iterbench.py --N $n --reps 3 > gpurun_out/r04p_iter$n.txt 2>&1 || exit 1
done &&
timeout -k 10 300 python -u bench.py > gpurun_out/r04p_bench_c2.json 2> gpurun_out/r04p_bench_c2.err &&
timeout -k 10 300 python -u bench.py --config c3 > gpurun_out/r04p_bench_c3.json 2> gpurun_out/r04p_bench_c3.err &&
bash tools/profile.sh r04pc3 --config c3 &&
bash tools/profile.sh r04p --config c2 &&
for v in prev16 cur16 prev16 cur16; do
  MPCQ_LIB_VARIANT=exp:$v timeout -k 10 180 python -u tools/iterbench.py --N 16 --reps 3 --batches 256 512 >> gpurun_out/r04p_ab16.txt 2>&1 || exit 1
done &&
for v in prev32 cur32 prev32 cur32; do
  MPCQ_LIB_VARIANT=exp:$v timeout -k 10 180 python -u tools/iterbench.py --N 32 --reps 3 --batches 256 >> gpurun_out/r04p_ab32.txt 2>&1 || exit 1
done
