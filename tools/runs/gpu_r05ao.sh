set -o pipefail
cd $GRAFT_REPO_ROOT
# r05ao: C3's HBM traffic with max-ilp scheduling at N = 32 (variant s_ilp32; the
# variant links the production build stamp, so its passes are read by hand, not merged
# into profiles/pmc_traffic.json), then the C3 line of each build, alternating
O=gpurun_out
MPCQ_LIB_VARIANT=exp:s_ilp32 bash tools/profile.sh r05ao_ilp32 --config c3 || exit 1
for r in 1 2; do
  for V in prod s_ilp32; do
    if [ $V = prod ]; then L=""; else L="exp:$V"; fi
    MPCQ_LIB_VARIANT=$L timeout -k 10 300 python -u bench.py --config c3 --cpu-sample 0 --companion 0 --certify 0 > $O/r05ao_c3_${V}_$r.json 2> $O/r05ao_c3_${V}_$r.err || exit 1
  done
done
