set -o pipefail
cd $GRAFT_REPO_ROOT
# r05a: HEAD after the CR/DC removal + the re-derived exit status beyond 16 stages:
# device count without HIP, the RCCL path at world 1, GPU suite, C2/C3 lines, stamped profiles
O=gpurun_out
python3 -c "import sys; sys.path.insert(0,'mpc-tsid_amd'); from mpcq import launch; import os; print('count_gpus', launch.count_gpus(), 'HIP_VISIBLE_DEVICES=%r' % os.environ.get('HIP_VISIBLE_DEVICES'), 'nodes', os.listdir(launch.KFD_TOPOLOGY) if os.path.isdir(launch.KFD_TOPOLOGY) else None)" > $O/r05a_count.txt 2>&1 &&
MPCQ_FORCE_DIST=1 MPCQ_DIST_BACKEND=nccl WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 timeout -k 10 300 python -u bench.py --gpus 1 --steps 5 --warmup 1 --companion 0 --cpu-sample 0 --certify 0 --restatement 64 --gather > $O/r05a_rccl_world1.json 2> $O/r05a_rccl_world1.err &&
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/r05a_pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r05a_smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/r05a_bench_c2.json 2> $O/r05a_bench_c2.err &&
timeout -k 10 300 python -u bench.py --config c3 > $O/r05a_bench_c3.json 2> $O/r05a_bench_c3.err &&
bash tools/profile.sh r05a --config c2 &&
bash tools/profile.sh r05ac3 --config c3
