set -o pipefail
cd $GRAFT_REPO_ROOT
# r05ab: LDS reads with exec-masked duplicate lanes (tools/ubench/lds_exec.hip), and the
# per-phase stamps of the current N = 16 build (nop elision in; st16 = stamps variant)
O=gpurun_out
timeout -k 10 120 tools/ubench/ldsx > $O/r05ab_ldsx.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:st16 timeout -k 10 200 python -u tools/stamps.py --N 16 --batch 256 --copies 0 > $O/r05ab_stamps16_alone.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:st16 timeout -k 10 200 python -u tools/stamps.py --N 16 --batch 512 --copies 0 > $O/r05ab_stamps16_co.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:st16 timeout -k 10 200 python -u tools/stamps.py --N 16 --batch 1024 > $O/r05ab_stamps16_batch.txt 2>&1
