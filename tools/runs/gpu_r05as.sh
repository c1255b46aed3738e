set -o pipefail
cd $GRAFT_REPO_ROOT
# r05as: as r05ar at more horizons (hi2 max-ilp, hd2 default), per
# iteration of each horizon's slowest trot instance, alternating
O=gpurun_out
for r in 1 2; do
  for N in 12 20 28 36 52 57; do
    for V in hd hi; do
      MPCQ_LIB_VARIANT=exp:${V}2 timeout -k 10 300 python -u tools/iterbench.py --N $N --reps 2 --batches 256 > $O/r05as_iter${N}_${V}_$r.txt 2>&1 || exit 1
    done
  done
done
