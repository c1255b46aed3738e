set -o pipefail
cd $GRAFT_REPO_ROOT
# r05x: the check's constant block read at the start of the DELTA iteration (ce,
# MPCQ_CK_EARLY) against after its sweep (hw = the current source), same box, alternating;
# check cost and per iteration at OSQP's interval 25
O=gpurun_out
for r in 1 2; do
  for V in hw16 ce16; do
    MPCQ_LIB_VARIANT=exp:$V timeout -k 10 200 python -u tools/checkcost.py --N 16 > $O/r05x_checkcost16_${V}_$r.txt 2>&1 || exit 1
    MPCQ_LIB_VARIANT=exp:$V timeout -k 10 200 python -u tools/iterbench.py --N 16 --reps 3 --batches 256 512 > $O/r05x_iter16_${V}_$r.txt 2>&1 || exit 1
  done
  for V in hw32 ce32; do
    MPCQ_LIB_VARIANT=exp:$V timeout -k 10 200 python -u tools/iterbench.py --N 32 --reps 3 --batches 256 > $O/r05x_iter32_${V}_$r.txt 2>&1 || exit 1
  done
done
