set -o pipefail
cd $GRAFT_REPO_ROOT
# r06b: HEAD with the gait-class dispatch order (MPCQ_FLAG_ORDER_BY_CLASS) -- the RCCL path at
# world 1 with the stdout redirect (one JSON line, dist.backend nccl), the GPU suite, C2 and
# the C5 shard with and without the class order (A/B on one box)
O=gpurun_out
MPCQ_FORCE_DIST=1 MPCQ_DIST_BACKEND=nccl WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 timeout -k 10 300 python -u bench.py --gpus 1 --steps 5 --warmup 1 --companion 0 --reference25 0 --cpu-sample 0 --certify 0 --restatement 64 --gather > $O/r06b_rccl_world1.json 2> $O/r06b_rccl_world1.err &&
python3 -c "
import json,sys
L=[l for l in open('$O/r06b_rccl_world1.json').read().splitlines() if l.strip()]
assert len(L)==1, L
d=json.loads(L[0]); print('rccl world1 stdout lines', len(L), 'dist', d['dist'], 'value', d['value'])
assert d['dist']['backend']=='nccl'
" > $O/r06b_rccl_check.txt 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/r06b_pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/r06b_bench_c2.json 2> $O/r06b_bench_c2.err &&
timeout -k 10 300 python -u bench.py --order-by-class 0 --companion 0 --reference25 0 --cpu-sample 0 --certify 0 --restatement 0 > $O/r06b_bench_c2_noorder.json 2> $O/r06b_bench_c2_noorder.err &&
timeout -k 10 300 python -u bench.py --config c5 --batch 4096 --companion 0 --reference25 0 --cpu-sample 0 --certify 0 --restatement 512 > $O/r06b_bench_c5_shard4096.json 2> $O/r06b_bench_c5_shard.err &&
timeout -k 10 300 python -u bench.py --config c5 --batch 4096 --order-by-class 0 --companion 0 --reference25 0 --cpu-sample 0 --certify 0 --restatement 0 > $O/r06b_bench_c5_shard4096_noorder.json 2> $O/r06b_bench_c5_shard_noorder.err &&
timeout -k 10 300 python -u bench.py --config c5 --steps 3 --warmup 1 --companion 0 --reference25 0 --cpu-sample 0 --certify 0 --restatement 512 > $O/r06b_bench_c5_1gpu.json 2> $O/r06b_bench_c5.err
