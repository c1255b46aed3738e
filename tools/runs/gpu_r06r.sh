set -o pipefail
cd $GRAFT_REPO_ROOT
# r06r: C3's slice length around r06q's best (1000 / 1200 / 1400, residual-ordered resumption),
# then slice once (an experiment, MPCQ_SLICE_ONCE=1: the resumed launch runs every suspended
# instance to its end) at 800 / 1200 / 1600
O=gpurun_out
T=r06r
L="--companion 0 --reference25 0 --cpu-sample 0 --certify 0 --restatement 1024"
for q in 1000 1200 1400; do
  timeout -k 10 240 python -u bench.py --config c3 $L --slice $q > $O/${T}_bench_c3_s$q.json 2> $O/${T}_bench_c3_s$q.err || exit 1
done
for q in 800 1200 1600; do
  MPCQ_SLICE_ONCE=1 timeout -k 10 240 python -u bench.py --config c3 $L --slice $q > $O/${T}_bench_c3_once_s$q.json 2> $O/${T}_bench_c3_once_s$q.err || exit 1
done
