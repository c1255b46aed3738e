set -o pipefail
cd $GRAFT_REPO_ROOT
# r05y: the inward sweep's half-1 hand-off by ds_bpermute issued a chain ahead plus a select
# (bp, MPCQ_SWEEP_BPERM) against v_permlane32_swap after the chain (hw = current), alternating
O=gpurun_out
for r in 1 2; do
  for V in hw16 bp16; do
    MPCQ_LIB_VARIANT=exp:$V timeout -k 10 200 python -u tools/iterbench.py --N 16 --reps 3 --batches 256 512 > $O/r05y_iter16_${V}_$r.txt 2>&1 || exit 1
  done
  for V in hw32 bp32; do
    MPCQ_LIB_VARIANT=exp:$V timeout -k 10 200 python -u tools/iterbench.py --N 32 --reps 3 --batches 256 > $O/r05y_iter32_${V}_$r.txt 2>&1 || exit 1
  done
done
MPCQ_LIB_VARIANT=exp:bp16 timeout -k 10 300 python -u bench.py --cpu-sample 0 --companion 0 > $O/r05y_bench_c2_bp16.json 2> $O/r05y_bench_c2_bp16.err
