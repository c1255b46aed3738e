set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
# per-phase cycles at N = 32 (C3) and N = 16, one copy of the slowest instance per CU, final source
MPCQ_LIB_VARIANT=exp:stv timeout -k 10 300 python -u tools/stamps.py --N 32 --batch 256 --copies 19 > $O/r03st_stamps32.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:stv timeout -k 10 300 python -u tools/stamps.py --N 16 --batch 256 --copies 0 > $O/r03st_stamps16.txt 2>&1
