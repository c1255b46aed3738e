set -o pipefail
cd $GRAFT_REPO_ROOT
# r05aa: the engine through nop_elide.py (then under tools/, base built with it off) (the asm blocks' opening s_nop 1 dropped
# where the schedule already separates them from their inputs) against the same source
# without the pass (base), alternating; digests must agree bit for bit
O=gpurun_out
for V in base nopel; do
  MPCQ_LIB_VARIANT=exp:$V timeout -k 10 200 python -u tools/variant_digest.py > $O/r05aa_digest_$V.txt 2>&1 || exit 1
done
for r in 1 2; do
  for V in base nopel; do
    MPCQ_LIB_VARIANT=exp:$V timeout -k 10 200 python -u tools/iterbench.py --N 16 --reps 3 --batches 256 512 > $O/r05aa_iter16_${V}_$r.txt 2>&1 || exit 1
    MPCQ_LIB_VARIANT=exp:$V timeout -k 10 200 python -u tools/iterbench.py --N 32 --reps 3 --batches 256 > $O/r05aa_iter32_${V}_$r.txt 2>&1 || exit 1
  done
done
for V in base nopel; do
  MPCQ_LIB_VARIANT=exp:$V timeout -k 10 300 python -u bench.py --cpu-sample 0 --companion 0 > $O/r05aa_bench_c2_$V.json 2> $O/r05aa_bench_c2_$V.err || exit 1
done
