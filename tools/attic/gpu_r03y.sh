set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
# r03y: is the check's cost its scratch reloads?  ckone = the check's constants as
# immediates (timing only), against tb (production); interleaved, twice
for r in 1 2; do for v in tb ckone; do
  MPCQ_LIB_VARIANT=exp:$v timeout -k 10 300 python -u tools/checkcost.py > $O/r03y_checkcost_${v}_$r.txt 2>&1 || exit 1
done; done
