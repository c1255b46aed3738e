set -o pipefail
cd $GRAFT_REPO_ROOT
# r05ae: the C3 batch (N = 32) under the scheduler strategies of r05ad: cur (default,
# production at N = 32), s_mmc (max-memory-clause), s_ilp (max-ilp), alternating
O=gpurun_out
for r in 1 2; do
  for V in cur s_mmc s_ilp; do
    MPCQ_LIB_VARIANT=exp:$V timeout -k 10 300 python -u bench.py --config c3 --cpu-sample 0 --companion 0 > $O/r05ae_c3_${V}_$r.json 2> $O/r05ae_c3_${V}_$r.err || exit 1
  done
done
