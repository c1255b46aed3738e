set -o pipefail
cd $GRAFT_REPO_ROOT
# r05g: u = F b_f formed behind the right-hand-side stores (kUfLate) against before
# (MPCQ_UF_EARLY), same box, alternating; N = 16 and N = 32
O=gpurun_out
for r in 1 2; do
  for V in ufe16 ufl16; do
    MPCQ_LIB_VARIANT=exp:$V timeout -k 10 200 python -u tools/iterbench.py --N 16 --reps 3 --batches 256 512 1024 > $O/r05g_iter16_${V}_$r.txt 2>&1 || exit 1
  done
  for V in ufe32 ufl32; do
    MPCQ_LIB_VARIANT=exp:$V timeout -k 10 200 python -u tools/iterbench.py --N 32 --reps 3 --batches 256 1024 > $O/r05g_iter32_${V}_$r.txt 2>&1 || exit 1
  done
done
MPCQ_LIB_VARIANT=exp:ufl16 timeout -k 10 300 python -u bench.py --cpu-sample 0 --companion 0 > $O/r05g_bench_c2_ufl16.json 2> $O/r05g_bench_c2_ufl16.err
