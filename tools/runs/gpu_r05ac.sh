set -o pipefail
cd $GRAFT_REPO_ROOT
# r05ac: the inward sweep's right-hand-side pair through bases of their own and the half-0
# add under an exec mask (bx, -DMPCQ_BEXEC) against the current source (cur), alternating
# (not kept: the variant added two laundered na-base pointers and an add_lo32() helper -- v_add_f64
# under s_mov_b32 exec_hi, 0 -- to ph_sweep_lag; 1.86-1.89 vs 1.80-1.82 us at N = 16, 2.985 vs
# 2.892 at N = 32, digests identical; the code was removed after this run)
O=gpurun_out
for V in cur bx; do
  MPCQ_LIB_VARIANT=exp:$V timeout -k 10 200 python -u tools/variant_digest.py > $O/r05ac_digest_$V.txt 2>&1 || exit 1
done
for r in 1 2; do
  for V in cur bx; do
    MPCQ_LIB_VARIANT=exp:$V timeout -k 10 200 python -u tools/iterbench.py --N 16 --reps 3 --batches 256 512 > $O/r05ac_iter16_${V}_$r.txt 2>&1 || exit 1
    MPCQ_LIB_VARIANT=exp:$V timeout -k 10 200 python -u tools/iterbench.py --N 32 --reps 3 --batches 256 > $O/r05ac_iter32_${V}_$r.txt 2>&1 || exit 1
  done
done
