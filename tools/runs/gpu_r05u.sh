set -o pipefail
cd $GRAFT_REPO_ROOT
# r05u: N = 64 per-iteration bisection: round 4's engine (260679a), r05a (496ff12), r05n
# (62d7d0c) and the current source, same box
O=gpurun_out
for V in r4_64 r5a_64 r5n_64 cur64; do
  MPCQ_LIB_VARIANT=exp:$V timeout -k 10 300 python -u tools/iterbench.py --N 64 --reps 2 --batches 32 256 > $O/r05u_iter64_$V.txt 2>&1 || exit 1
done
