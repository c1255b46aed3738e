set -o pipefail
cd $GRAFT_REPO_ROOT
# r06n: C3's slice length (1200 / 2000 / 2400 / 2800 iterations; r06m: 400 / 800 / 1600 and
# unsliced), the nested-dissection variant A/B (its library rebuilt with mpcq_set_slice), C2 sliced
O=gpurun_out
T=r06n
L="--companion 0 --reference25 0 --cpu-sample 0 --certify 0 --restatement 1024"
for q in 1200 2000 2400 2800; do
  timeout -k 10 240 python -u bench.py --config c3 $L --slice $q > $O/${T}_bench_c3_s$q.json 2> $O/${T}_bench_c3_s$q.err || exit 1
done
timeout -k 10 240 python -u bench.py --config c3 $L --slice 1600 > $O/${T}_bench_c3_s1600.json 2> $O/${T}_bench_c3_s1600.err &&
timeout -k 10 240 python -u tools/iterbench.py --N 32 --batches 256 > $O/${T}_iter32_prod.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:ndv timeout -k 10 240 python -u tools/iterbench.py --N 32 --batches 256 > $O/${T}_iter32_ndv.txt 2>&1 &&
timeout -k 10 120 python -u tools/stamps.py --N 32 --batch 256 --copies 0 > $O/${T}_stamps32_prod.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:st32ndv timeout -k 10 120 python -u tools/stamps.py --N 32 --batch 256 --copies 0 --nd > $O/${T}_stamps32_ndv.txt 2>&1
# slicing at 16 stages (an experiment: libmpcq_sl16.so, -DMPCQ_SLICE16, MPCQ_SLICE16=1 lets the
# host slice N = 16): C2 unsliced (production), then sliced at 1200 / 1600 / 2000 / 2400
[ $? -eq 0 ] &&
timeout -k 10 240 python -u bench.py $L > $O/${T}_bench_c2_prod.json 2> $O/${T}_bench_c2_prod.err &&
for q in 1200 1600 2000 2400; do
  MPCQ_SLICE16=1 MPCQ_LIB_VARIANT=exp:sl16 timeout -k 10 240 python -u bench.py $L --slice $q > $O/${T}_bench_c2_sl16_s$q.json 2> $O/${T}_bench_c2_sl16_s$q.err || exit 1
done
