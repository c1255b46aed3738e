set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
# r03pre2: the whole constant block read once in the last iteration before the check
# (update_info and the products pass use it too) vs pre (infeas_cheap's part only)
for r in 1 2 3; do
  MPCQ_LIB_VARIANT=exp:pre timeout -k 10 300 python -u tools/checkcost.py > $O/r03pre2_checkcost_pre_$r.txt 2>&1 &&
  MPCQ_LIB_VARIANT=exp:pre2 timeout -k 10 300 python -u tools/checkcost.py > $O/r03pre2_checkcost_pre2_$r.txt 2>&1 || exit 1
done
MPCQ_LIB_VARIANT=exp:pre timeout -k 10 300 python -u tools/iterbench.py --reps 3 > $O/r03pre2_iter_pre.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:pre2 timeout -k 10 300 python -u tools/iterbench.py --reps 3 > $O/r03pre2_iter_pre2.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/r03pre2_pytest_gpu.log 2>&1
