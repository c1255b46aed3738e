set -o pipefail
cd $GRAFT_REPO_ROOT
# r05ad: machine-scheduler strategies at N = 16 / 32 (per iteration, C2's slowest instance):
# cur = default, s_ilp = max-ilp (production at N = 16), s_mmc = max-memory-clause,
# s_trk = default with -amdgpu-use-amdgpu-trackers=1 (iterative-ilp crashes the compiler)
O=gpurun_out
for r in 1 2; do
  for V in cur s_ilp s_mmc s_trk; do
    MPCQ_LIB_VARIANT=exp:$V timeout -k 10 200 python -u tools/iterbench.py --N 16 --reps 3 --batches 256 512 > $O/r05ad_iter16_${V}_$r.txt 2>&1 || exit 1
    MPCQ_LIB_VARIANT=exp:$V timeout -k 10 200 python -u tools/iterbench.py --N 32 --reps 3 --batches 256 > $O/r05ad_iter32_${V}_$r.txt 2>&1 || exit 1
  done
done
