set -o pipefail
cd $GRAFT_REPO_ROOT
# r05av: on top of max-ilp at N = 32 / 48 / 64 (m0 = production flags): m1 adds
# -amdgpu-disable-unclustered-high-rp-reschedule, m2 -amdgpu-disable-clustered-low-occupancy-reschedule;
# per iteration with 256 in flight, alternating
O=gpurun_out
for r in 1 2; do
  for N in 32 48 64; do
    for V in m0 m1 m2; do
      MPCQ_LIB_VARIANT=exp:$V timeout -k 10 300 python -u tools/iterbench.py --N $N --reps 2 --batches 256 > $O/r05av_iter${N}_${V}_$r.txt 2>&1 || exit 1
    done
  done
done
