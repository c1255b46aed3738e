set -o pipefail
cd $GRAFT_REPO_ROOT
# r05h: Gauss-Jordan with lazy pivot rows (kGjLazy) against the normalised form
# (MPCQ_GJ_NORM): factorisation cycles (tools/factime.py), C2 / C4 / C3 launches with
# the oracle restatement's status / iteration agreement
O=gpurun_out
for r in 1 2; do
  for V in n l; do
    MPCQ_LIB_VARIANT=exp:ft${V}16 timeout -k 10 120 python -u tools/factime.py 16 > $O/r05h_factime16_ft${V}_$r.txt 2>&1 || exit 1
    MPCQ_LIB_VARIANT=exp:ft${V}32 timeout -k 10 120 python -u tools/factime.py 32 > $O/r05h_factime32_ft${V}_$r.txt 2>&1 || exit 1
  done
done
for V in gjn16 gjl16; do
  MPCQ_LIB_VARIANT=exp:$V timeout -k 10 300 python -u bench.py --cpu-sample 0 --companion 0 > $O/r05h_bench_c2_$V.json 2> $O/r05h_bench_c2_$V.err || exit 1
  MPCQ_LIB_VARIANT=exp:$V timeout -k 10 300 python -u bench.py --config c4 --cpu-sample 0 --companion 0 --certify 0 --restatement 0 > $O/r05h_bench_c4_$V.json 2> $O/r05h_bench_c4_$V.err || exit 1
done
for V in gjn32 gjl32; do
  MPCQ_LIB_VARIANT=exp:$V timeout -k 10 400 python -u bench.py --config c3 --cpu-sample 0 --companion 0 --certify 0 > $O/r05h_bench_c3_$V.json 2> $O/r05h_bench_c3_$V.err || exit 1
done
