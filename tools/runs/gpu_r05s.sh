set -o pipefail
cd $GRAFT_REPO_ROOT
# r05s: hardware max / clamp (no canonicalisation) on top of the rhs cuts (hw) against the rhs
# cuts alone (bo), same box, alternating; check cost of both
O=gpurun_out
for r in 1 2; do
  for V in bo16 hw16; do
    MPCQ_LIB_VARIANT=exp:$V timeout -k 10 200 python -u tools/iterbench.py --N 16 --reps 3 --batches 256 512 > $O/r05s_iter16_${V}_$r.txt 2>&1 || exit 1
  done
  for V in bo32 hw32; do
    MPCQ_LIB_VARIANT=exp:$V timeout -k 10 200 python -u tools/iterbench.py --N 32 --reps 3 --batches 256 > $O/r05s_iter32_${V}_$r.txt 2>&1 || exit 1
  done
done
for V in bo16 hw16; do
  MPCQ_LIB_VARIANT=exp:$V timeout -k 10 200 python -u tools/checkcost.py --N 16 > $O/r05s_checkcost16_$V.txt 2>&1 || exit 1
done
MPCQ_LIB_VARIANT=exp:hw16 timeout -k 10 300 python -u bench.py --cpu-sample 0 --companion 0 > $O/r05s_bench_c2_hw16.json 2> $O/r05s_bench_c2_hw16.err
