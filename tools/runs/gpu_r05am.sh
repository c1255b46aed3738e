set -o pipefail
cd $GRAFT_REPO_ROOT
# r05am: age-based wave priorities (-DMPCQ_AGEPRIO=T: past T iterations an instance's sweep
# runs at s_setprio 3 and its stage work at 2, younger ones at 1 / 0) against the production
# flags (k0), N = 16: C2 alternating, then C4 / C5 on one GPU; digests must agree
# (not kept: C2 131.6-132.2 k against 134.2-134.4 k, C4 232.9 / 234.9 k against 238.5 k, C5
# 297.5 / 300.3 k against 304.3 k, digests identical; the MPCQ_AGEPRIO code was removed)
O=gpurun_out
for V in k0 ap1000; do
  MPCQ_LIB_VARIANT=exp:$V timeout -k 10 200 python -u tools/variant_digest.py --N 16 > $O/r05am_digest_$V.txt 2>&1 || exit 1
done
B="--cpu-sample 0 --companion 0 --certify 0"
for r in 1 2; do
  for V in k0 ap1000 ap400; do
    MPCQ_LIB_VARIANT=exp:$V timeout -k 10 300 python -u bench.py $B > $O/r05am_c2_${V}_$r.json 2> $O/r05am_c2_${V}_$r.err || exit 1
  done
done
for V in k0 ap1000 ap400; do
  MPCQ_LIB_VARIANT=exp:$V timeout -k 10 300 python -u bench.py --config c4 --steps 3 --warmup 1 $B > $O/r05am_c4_${V}.json 2> $O/r05am_c4_${V}.err || exit 1
  MPCQ_LIB_VARIANT=exp:$V timeout -k 10 300 python -u bench.py --config c5 --steps 3 --warmup 1 $B > $O/r05am_c5_${V}.json 2> $O/r05am_c5_${V}.err || exit 1
done
