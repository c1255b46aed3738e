set -o pipefail
cd $GRAFT_REPO_ROOT
# r05v: beyond 32 stages with the exit status carried in a register again (xr: kXstRe off)
# against the current source, N = 48 / 64, same box
O=gpurun_out
for V in cur64 xr64; do
  MPCQ_LIB_VARIANT=exp:$V timeout -k 10 300 python -u tools/iterbench.py --N 64 --reps 2 --batches 32 256 > $O/r05v_iter64_$V.txt 2>&1 || exit 1
done
for V in cur48 xr64; do
  MPCQ_LIB_VARIANT=exp:$V timeout -k 10 300 python -u tools/iterbench.py --N 48 --reps 2 --batches 32 256 > $O/r05v_iter48_$V.txt 2>&1 || exit 1
done
