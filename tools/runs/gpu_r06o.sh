set -o pipefail
cd $GRAFT_REPO_ROOT
# r06o: slicing at 16 stages (an experiment: libmpcq_sl16.so, -DMPCQ_SLICE16; MPCQ_SLICE16=1 lets
# the host slice N = 16): C2 unsliced (production), then sliced at 1200 / 1600 / 2000 / 2400; C5's
# rank shard unsliced / sliced at 1600 (r06n's tail, which stopped at the stamps library)
O=gpurun_out
T=r06o
L="--companion 0 --reference25 0 --cpu-sample 0 --certify 0 --restatement 1024"
timeout -k 10 240 python -u bench.py $L > $O/${T}_bench_c2_prod.json 2> $O/${T}_bench_c2_prod.err || exit 1
for q in 1200 1600 2000 2400; do
  MPCQ_SLICE16=1 MPCQ_LIB_VARIANT=exp:sl16 timeout -k 10 240 python -u bench.py $L --slice $q > $O/${T}_bench_c2_sl16_s$q.json 2> $O/${T}_bench_c2_sl16_s$q.err || exit 1
done
timeout -k 10 240 python -u bench.py --config c5 --batch 4096 $L > $O/${T}_bench_c5s_prod.json 2> $O/${T}_bench_c5s_prod.err &&
MPCQ_SLICE16=1 MPCQ_LIB_VARIANT=exp:sl16 timeout -k 10 240 python -u bench.py --config c5 --batch 4096 $L --slice 1600 > $O/${T}_bench_c5s_sl16_s1600.json 2> $O/${T}_bench_c5s_sl16.err &&
MPCQ_SLICE16=1 MPCQ_LIB_VARIANT=exp:sl16 timeout -k 10 240 python -u bench.py --config c5 --batch 4096 $L --slice 800 > $O/${T}_bench_c5s_sl16_s800.json 2> $O/${T}_bench_c5s_sl16_800.err
