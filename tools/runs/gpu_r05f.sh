set -o pipefail
cd $GRAFT_REPO_ROOT
# r05f: occupancy experiment: the 16-stage kernel in the beyond-32
# layout at 3 / 4 instances per CU (exp:occ3 / exp:occ4) against the production build
O=gpurun_out
for V in prod occ3 occ4; do
  if [ $V = prod ]; then unset MPCQ_LIB_VARIANT; else export MPCQ_LIB_VARIANT=exp:$V; fi
  timeout -k 10 300 python -u tools/iterbench.py --N 16 --reps 3 --batches 256 512 768 1024 > $O/r05f_iter16_$V.txt 2>&1 || exit 1
  for C in c2 c4 c5; do
    timeout -k 10 300 python -u bench.py --config $C --certify 0 --cpu-sample 0 --companion 0 > $O/r05f_bench_${C}_$V.json 2> $O/r05f_bench_${C}_$V.err || exit 1
  done
done
