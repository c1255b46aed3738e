set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
# r03big: beyond 32 stages, the check constants from the private block read ahead (bigck)
# vs from registers (bigprod = the final source); N = 48 / 56, interleaved, twice
for r in 1 2; do for v in bigprod bigck; do
  MPCQ_LIB_VARIANT=exp:$v timeout -k 10 300 python -u tools/iterbench.py --N 48 --reps 2 > $O/r03big_iter48_${v}_$r.txt 2>&1 &&
  MPCQ_LIB_VARIANT=exp:$v timeout -k 10 300 python -u tools/iterbench.py --N 56 --reps 2 > $O/r03big_iter56_${v}_$r.txt 2>&1 || exit 1
done; done
