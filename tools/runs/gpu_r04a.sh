set -o pipefail
cd $GRAFT_REPO_ROOT
# r04a: round 4's first box -- GPU suite (C4 full size + rank shard, N = 49 / 50), smoke,
# the C2 line (osqp_interval_band), bench.py's own 2-rank launch (gloo rehearsal on one
# card), and lines at the per-rank shard sizes of C4 (8192) and C5 (4096)
T=r04a
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/${T}_pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/${T}_bench_c2.json 2> $O/${T}_bench_c2.err &&
MPCQ_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 > $O/${T}_rehearsal_2rank_self.json 2> $O/${T}_rehearsal_2rank_self.err &&
timeout -k 10 300 python -u bench.py --config c4 --batch 8192 --companion 0 --cpu-sample 0 --certify 0 --restatement 512 > $O/${T}_bench_c4_shard8192.json 2> $O/${T}_bench_c4_shard.err &&
timeout -k 10 300 python -u bench.py --config c5 --batch 4096 --companion 0 --cpu-sample 0 --certify 0 --restatement 512 > $O/${T}_bench_c5_shard4096.json 2> $O/${T}_bench_c5_shard.err &&
timeout -k 10 300 python -u bench.py --config c4 --steps 3 --warmup 1 --companion 0 --cpu-sample 0 --certify 0 --restatement 512 > $O/${T}_bench_c4_1gpu.json 2> $O/${T}_bench_c4.err &&
timeout -k 10 300 python -u bench.py --config c5 --steps 3 --warmup 1 --companion 0 --cpu-sample 0 --certify 0 --restatement 512 > $O/${T}_bench_c5_1gpu.json 2> $O/${T}_bench_c5.err
