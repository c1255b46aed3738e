set -o pipefail
cd $GRAFT_REPO_ROOT
# r06v: the slicing tests with N = 64 added (the workspace layouts beyond 48 / 49 stages), the
# RCCL path at world 1 on the final build (stdout one JSON line, backend nccl)
O=gpurun_out
T=r06v
timeout -k 10 400 python -u -m pytest tests/test_gpu_slice.py -x -v --timeout 240 --timeout-method thread > $O/${T}_pytest_slice.log 2>&1 &&
MPCQ_FORCE_DIST=1 MPCQ_DIST_BACKEND=nccl WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 timeout -k 10 300 python -u bench.py --gpus 1 --steps 5 --warmup 1 --companion 0 --reference25 0 --cpu-sample 0 --certify 0 --restatement 64 --gather > $O/${T}_rccl_world1.json 2> $O/${T}_rccl_world1.err &&
python3 -c "
import json
L=[l for l in open('$O/${T}_rccl_world1.json').read().splitlines() if l.strip()]
assert len(L)==1, L
d=json.loads(L[0]); print('rccl world1: stdout lines', len(L), 'dist', d['dist'], 'value', d['value'], 'solved', d['solved_fraction'])
assert d['dist']['backend']=='nccl'
" > $O/${T}_rccl_check.txt 2>&1
