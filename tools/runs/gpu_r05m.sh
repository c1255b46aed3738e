set -o pipefail
cd $GRAFT_REPO_ROOT
# r05m: the sweep's step-1 rows read at the start of the right-hand-side phase
# (MPCQ_ROW1_EARLY) against after its stores, same box, alternating
O=gpurun_out
for r in 1 2; do
  for V in r1p16 r1e16; do
    MPCQ_LIB_VARIANT=exp:$V timeout -k 10 200 python -u tools/iterbench.py --N 16 --reps 3 --batches 256 512 > $O/r05m_iter16_${V}_$r.txt 2>&1 || exit 1
  done
  for V in r1p32 r1e32; do
    MPCQ_LIB_VARIANT=exp:$V timeout -k 10 200 python -u tools/iterbench.py --N 32 --reps 3 --batches 256 > $O/r05m_iter32_${V}_$r.txt 2>&1 || exit 1
  done
done
