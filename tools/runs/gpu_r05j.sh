set -o pipefail
cd $GRAFT_REPO_ROOT
# r05j: drift against the oracle (tools/drift.py) with the lazy and the normalised
# Gauss-Jordan pivot rows, N = 16 / 48 / 64
O=gpurun_out
for V in gjnh gjlh; do
  MPCQ_LIB_VARIANT=exp:$V timeout -k 10 400 python -u tools/drift.py --horizons 16 48 64 > $O/r05j_drift_$V.txt 2>&1 || exit 1
done
