set -o pipefail
cd $GRAFT_REPO_ROOT
# r05ar: max-ilp scheduling at other horizons (hi) against the default strategy (hd), per
# iteration of each horizon's slowest trot instance, alternating
O=gpurun_out
for r in 1 2; do
  for N in 8 24 40 48 64; do
    for V in hd hi; do
      MPCQ_LIB_VARIANT=exp:$V timeout -k 10 300 python -u tools/iterbench.py --N $N --reps 2 --batches 256 > $O/r05ar_iter${N}_${V}_$r.txt 2>&1 || exit 1
    done
  done
done
