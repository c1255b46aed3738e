set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
# r03x: the check's row maxima by a transposing butterfly (tb), + ratio maxima only at
# adaptive-rho checks (rs), against the round's final source (base); same box
for v in base tb rs; do
  MPCQ_LIB_VARIANT=exp:$v timeout -k 10 300 python -u tools/checkcost.py > $O/r03x_checkcost_$v.txt 2>&1 &&
  MPCQ_LIB_VARIANT=exp:$v timeout -k 10 300 python -u tools/iterbench.py --reps 3 > $O/r03x_iter16_$v.txt 2>&1 || exit 1
done
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/r03x_pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/r03x_bench_c2.json 2> $O/r03x_bench_c2.err &&
timeout -k 10 300 python -u bench.py --config c3 > $O/r03x_bench_c3.json 2> $O/r03x_bench_c3.err
