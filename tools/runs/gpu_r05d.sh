set -o pipefail
cd $GRAFT_REPO_ROOT
# r05d: per-phase cycles of the explicit-inverse iteration, stage wave 0 and helper wave 4,
# C2's slowest instance alone (256 copies) and the C2 batch
O=gpurun_out
MPCQ_LIB_VARIANT=exp:kist0 timeout -k 10 120 python -u tools/stamps.py --ki --copies 0 --batch 256 > $O/r05d_stamps_w0.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:kist4 timeout -k 10 120 python -u tools/stamps.py --ki --copies 0 --batch 256 > $O/r05d_stamps_w4.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:kist0 timeout -k 10 120 python -u tools/stamps.py --ki --batch 1024 > $O/r05d_stamps_w0_c2.txt 2>&1
