set -o pipefail
cd $GRAFT_REPO_ROOT
# r05p: right-hand-side phase instruction cuts (MPCQ_COLF_FOLD: colF's row broadcasts folded
# into v_fmac_f64_dpp; MPCQ_RHS_NOLAUNDER: no per-iteration pointer laundering), same box,
# alternating; then C2 parity on the combined build
O=gpurun_out
for r in 1 2; do
  for V in b16 cf16 nl16 bo16; do
    MPCQ_LIB_VARIANT=exp:$V timeout -k 10 200 python -u tools/iterbench.py --N 16 --reps 3 --batches 256 512 > $O/r05p_iter16_${V}_$r.txt 2>&1 || exit 1
  done
  for V in b32 bo32; do
    MPCQ_LIB_VARIANT=exp:$V timeout -k 10 200 python -u tools/iterbench.py --N 32 --reps 3 --batches 256 > $O/r05p_iter32_${V}_$r.txt 2>&1 || exit 1
  done
done
MPCQ_LIB_VARIANT=exp:bo16 timeout -k 10 300 python -u bench.py --cpu-sample 0 --companion 0 > $O/r05p_bench_c2_bo16.json 2> $O/r05p_bench_c2_bo16.err
