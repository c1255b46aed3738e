set -o pipefail
cd $GRAFT_REPO_ROOT
# r05q: the right-hand-side cuts (bo = colF fold + no rhs laundering) against the base, with
# the check's laundering dropped too (fc), and without the colF fold (nc); same box, alternating
O=gpurun_out
for r in 1 2; do
  for V in b16 bo16 fc16 nc16; do
    MPCQ_LIB_VARIANT=exp:$V timeout -k 10 200 python -u tools/iterbench.py --N 16 --reps 3 --batches 256 512 > $O/r05q_iter16_${V}_$r.txt 2>&1 || exit 1
  done
  for V in b32 bo32 fc32 nc32; do
    MPCQ_LIB_VARIANT=exp:$V timeout -k 10 200 python -u tools/iterbench.py --N 32 --reps 3 --batches 256 > $O/r05q_iter32_${V}_$r.txt 2>&1 || exit 1
  done
done
for V in b16 bo16 fc16; do
  MPCQ_LIB_VARIANT=exp:$V timeout -k 10 300 python -u bench.py --cpu-sample 0 --companion 0 --certify 0 --restatement 0 > $O/r05q_bench_c2_$V.json 2> $O/r05q_bench_c2_$V.err || exit 1
done
