set -o pipefail
cd $GRAFT_REPO_ROOT
# r05l: where the right-hand-side barrier's wait goes (stamps of waves 0 / 1 / 3, the own
# LDS wait split from the barrier: bucket 12), C2's slowest instance alone (256 copies)
O=gpurun_out
for V in stw0 stw1 stw3; do
  MPCQ_LIB_VARIANT=exp:$V timeout -k 10 120 python -u tools/stamps.py --copies 0 --batch 256 > $O/r05l_stamps_$V.txt 2>&1 || exit 1
done
