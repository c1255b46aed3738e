set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
# r03o: per-horizon register-allocation variants beyond 32 stages (tools/bigsweep.py)
timeout -k 10 300 python -u tools/bigsweep.py > $O/r03o_sweep_prod.txt 2>&1 &&
timeout -k 10 300 env MPCQ_LIB_VARIANT=exp:frheld python -u tools/bigsweep.py > $O/r03o_sweep_frheld.txt 2>&1 &&
timeout -k 10 300 env MPCQ_LIB_VARIANT=exp:zcheld python -u tools/bigsweep.py > $O/r03o_sweep_zcheld.txt 2>&1 &&
timeout -k 10 300 env MPCQ_LIB_VARIANT=exp:bothheld python -u tools/bigsweep.py > $O/r03o_sweep_bothheld.txt 2>&1
