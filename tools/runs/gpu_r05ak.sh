set -o pipefail
cd $GRAFT_REPO_ROOT
# r05ak: the inward sweep's na right-hand sides through laundered bases of their own (sb,
# -DMPCQ_SEPB: two ds_read_b64 at immediate offsets per step instead of an address add and
# a ds_read2st64) against the production flags (k0), N = 16, alternating; digests must agree
# (not kept: 1.744-1.752 against 1.716-1.725 us alone, 2.094-2.101 against 2.058-2.065 at two
# per CU, digests identical; the MPCQ_SEPB code was removed after this run)
O=gpurun_out
for V in k0 sb; do
  MPCQ_LIB_VARIANT=exp:$V timeout -k 10 200 python -u tools/variant_digest.py --N 16 > $O/r05ak_digest_$V.txt 2>&1 || exit 1
done
for r in 1 2 3; do
  for V in k0 sb; do
    MPCQ_LIB_VARIANT=exp:$V timeout -k 10 200 python -u tools/iterbench.py --N 16 --reps 3 --batches 256 512 > $O/r05ak_iter16_${V}_$r.txt 2>&1 || exit 1
  done
done
