set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
# r03z: the check's constants (E, the dynamics bound, the infeasibility tolerances
# included) read in one batch per check phase; against tb (the butterfly alone)
for r in 1 2; do
  MPCQ_LIB_VARIANT=exp:tb timeout -k 10 300 python -u tools/checkcost.py > $O/r03z_checkcost_tb_$r.txt 2>&1 &&
  timeout -k 10 300 python -u tools/checkcost.py > $O/r03z_checkcost_new_$r.txt 2>&1 || exit 1
done
timeout -k 10 300 python -u tools/iterbench.py --reps 3 > $O/r03z_iter16.txt 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/r03z_pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/r03z_bench_c2.json 2> $O/r03z_bench_c2.err &&
timeout -k 10 300 python -u bench.py --config c3 > $O/r03z_bench_c3.json 2> $O/r03z_bench_c3.err
