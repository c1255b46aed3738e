set -o pipefail
cd $GRAFT_REPO_ROOT
# r05aj: LLVM scheduling knobs on top of max-ilp at N = 16 (per iteration, C2's slowest
# instance, alternating): k0 = production flags; k1 -amdgpu-disable-unclustered-high-rp-reschedule;
# k2 -amdgpu-disable-clustered-low-occupancy-reschedule; k3 -misched-cluster=false;
# k4 -enable-post-misched=false; k5 -misched-postra-direction=bottomup
O=gpurun_out
for r in 1 2; do
  for V in k0 k1 k2 k3 k4 k5; do
    MPCQ_LIB_VARIANT=exp:$V timeout -k 10 200 python -u tools/iterbench.py --N 16 --reps 3 --batches 256 512 > $O/r05aj_iter16_${V}_$r.txt 2>&1 || exit 1
  done
done
