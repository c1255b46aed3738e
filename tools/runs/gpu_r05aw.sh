set -o pipefail
cd $GRAFT_REPO_ROOT
# r05aw: on top of max-ilp at N = 16 (b0 = production flags): b1 -amdgpu-schedule-metric-bias=0,
# b2 -amdgpu-schedule-metric-bias=100, b3 -misched-postra-direction=bidirectional; per
# iteration on C2's slowest instance alone / two per CU, alternating (b1 and b2 disassemble
# identical to b0 -- asmpass/codeobj.py -- so only b3 runs)
O=gpurun_out
for r in 1 2; do
  for V in b0 b3; do
    MPCQ_LIB_VARIANT=exp:$V timeout -k 10 200 python -u tools/iterbench.py --N 16 --reps 3 --batches 256 512 > $O/r05aw_iter16_${V}_$r.txt 2>&1 || exit 1
  done
done
