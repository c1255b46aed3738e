# Every bench line of DESIGN.md §5 plus the rocprof passes, tagged: bash tools/bench_all.sh r04f
# (the headline mode is OSQP as MPC.py configures it; each qp line carries the polish=2 companion)
set -o pipefail
T=${1:?tag}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd $R
timeout -k 10 300 python -u bench.py > $O/${T}_bench_c2.json 2> $O/${T}_bench_c2.err &&
timeout -k 10 300 python -u bench.py --config c3 > $O/${T}_bench_c3.json 2> $O/${T}_bench_c3.err &&
timeout -k 10 240 python -u bench.py --config c1 > $O/${T}_bench_c1.json 2> $O/${T}_bench_c1.err &&
timeout -k 10 300 python -u bench.py --config c4 --steps 3 --warmup 1 > $O/${T}_bench_c4_1gpu.json 2> $O/${T}_bench_c4.err &&
timeout -k 10 300 python -u bench.py --config c5 --steps 3 --warmup 1 > $O/${T}_bench_c5_1gpu.json 2> $O/${T}_bench_c5.err &&
timeout -k 10 300 python -u bench.py --config c4 --batch 8192 --companion 0 --cpu-sample 0 --certify 0 --restatement 512 > $O/${T}_bench_c4_shard8192.json 2> $O/${T}_bench_c4_shard.err &&
timeout -k 10 300 python -u bench.py --config c5 --batch 4096 --companion 0 --cpu-sample 0 --certify 0 --restatement 512 > $O/${T}_bench_c5_shard4096.json 2> $O/${T}_bench_c5_shard.err &&
MPCQ_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --companion 0 --cpu-sample 0 --certify 0 > $O/${T}_rehearsal_2rank_self.json 2> $O/${T}_rehearsal_2rank_self.err &&
timeout -k 10 300 python -u bench.py --mode tick --steps 20 --warmup 4 > $O/${T}_bench_tick_c2.json 2> $O/${T}_bench_tick_c2.err &&
timeout -k 10 300 python -u bench.py --mode plan --cpu-sample 4096 > $O/${T}_bench_plan.json 2> $O/${T}_bench_plan.err &&
bash tools/profile.sh $T --config c2 &&
bash tools/profile.sh ${T}c3 --config c3
