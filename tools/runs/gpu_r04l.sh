set -o pipefail
cd $GRAFT_REPO_ROOT
# r04l: the factorisation's couplings read as column pairs -- GPU suite, factorisation
# cycles (FACTIME builds, old / new source), same-box bench A/B at N = 16 (variants old / new)
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04l_pytest_gpu.log 2>&1 &&
for v in ftold ftnew; do
  for n in 16 32; do
    MPCQ_LIB_VARIANT=exp:$v timeout -k 10 120 python -u tools/factime.py $n > gpurun_out/r04l_factime${n}_$v.txt 2>&1 || exit 1
  done
done &&
for v in old new old new; do
  MPCQ_LIB_VARIANT=exp:$v timeout -k 10 300 python -u bench.py --config c4 --steps 3 --warmup 1 --companion 0 --cpu-sample 0 --certify 0 --restatement 0 >> gpurun_out/r04l_bench_c4_ab.txt 2>> gpurun_out/r04l_bench_c4_ab.err || exit 1
  MPCQ_LIB_VARIANT=exp:$v timeout -k 10 300 python -u bench.py --companion 0 --cpu-sample 0 --certify 0 --restatement 0 >> gpurun_out/r04l_bench_c2_ab.txt 2>> gpurun_out/r04l_bench_c2_ab.err || exit 1
done
