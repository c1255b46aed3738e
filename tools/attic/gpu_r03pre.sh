set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
# r03pre: the check's constant block read in the last iteration before the check (behind
# the force recovery / update) vs the final build; interleaved, three times
for r in 1 2 3; do
  timeout -k 10 300 python -u tools/checkcost.py > $O/r03pre_checkcost_prod_$r.txt 2>&1 &&
  MPCQ_LIB_VARIANT=exp:pre timeout -k 10 300 python -u tools/checkcost.py > $O/r03pre_checkcost_pre_$r.txt 2>&1 || exit 1
done
timeout -k 10 300 python -u tools/iterbench.py --reps 3 > $O/r03pre_iter_prod.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:pre timeout -k 10 300 python -u tools/iterbench.py --reps 3 > $O/r03pre_iter_pre.txt 2>&1
