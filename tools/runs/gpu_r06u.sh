set -o pipefail
cd $GRAFT_REPO_ROOT
# r06u: slicing at 16 stages again, now resumed once residual-first (an experiment:
# libmpcq_sl16.so = -DMPCQ_SLICE16 with max-ilp, MPCQ_SLICE16=1 lets the host slice N = 16):
# C2 and the C5 shard unsliced (the variant) and at 800 / 1200 / 1600 / 2000; per iteration of
# the variant against production
O=gpurun_out
T=r06u
L="--companion 0 --reference25 0 --cpu-sample 0 --certify 0 --restatement 1024"
V="MPCQ_SLICE16=1 MPCQ_LIB_VARIANT=exp:sl16"
timeout -k 10 240 python -u tools/iterbench.py --N 16 --batches 256 > $O/${T}_iter16_prod.txt 2>&1 &&
env $V timeout -k 10 240 python -u tools/iterbench.py --N 16 --batches 256 > $O/${T}_iter16_sl16.txt 2>&1 &&
env $V timeout -k 10 240 python -u bench.py $L --slice 0 > $O/${T}_bench_c2_sl16_s0.json 2> $O/${T}_bench_c2_s0.err || exit 1
for q in 800 1200 1600 2000; do
  env $V timeout -k 10 240 python -u bench.py $L --slice $q > $O/${T}_bench_c2_sl16_s$q.json 2> $O/${T}_bench_c2_s$q.err || exit 1
done
for q in 0 600 800 1200; do
  env $V timeout -k 10 240 python -u bench.py --config c5 --batch 4096 $L --slice $q > $O/${T}_bench_c5s_sl16_s$q.json 2> $O/${T}_bench_c5s_s$q.err || exit 1
done
