set -o pipefail
cd $GRAFT_REPO_ROOT
# r06f (1 of 3): the round's final build -- smoke, the HEAD RCCL path at world 1 (stdout = one JSON
# line, dist.backend nccl), the whole GPU suite
O=gpurun_out
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/r06f_smoke.log 2>&1 &&
MPCQ_FORCE_DIST=1 MPCQ_DIST_BACKEND=nccl WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 timeout -k 10 300 python -u bench.py --gpus 1 --steps 5 --warmup 1 --companion 0 --reference25 0 --cpu-sample 0 --certify 0 --restatement 64 --gather > $O/r06f_rccl_world1.json 2> $O/r06f_rccl_world1.err &&
python3 -c "
import json
L=[l for l in open('$O/r06f_rccl_world1.json').read().splitlines() if l.strip()]
assert len(L)==1, L
d=json.loads(L[0]); print('rccl world1: stdout lines', len(L), 'dist', d['dist'], 'value', d['value'], 'solved', d['solved_fraction'])
assert d['dist']['backend']=='nccl'
" > $O/r06f_rccl_check.txt 2>&1 &&
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/r06f_pytest_gpu.log 2>&1
