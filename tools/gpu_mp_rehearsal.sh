#!/bin/bash
# bench.py's N > 1 path on a one-GPU box: 2 ranks launched exactly as the driver
# launches N GPUs (torch.distributed.run), sharing the card, collectives over gloo
# (MPCQ_DIST_BACKEND=gloo).  Checks that every rank runs the HIP engine and rank 0
# prints one line with n_gpus = 2; the numbers are not a scaling measurement.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
T=${1:-mp}
cd $R
export MPCQ_DIST_BACKEND=gloo
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 > $O/${T}_mp_qp.json 2> $O/${T}_mp_qp.err &&
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29532 bench.py --gpus 2 --steps 3 --warmup 1 --config c5 --batch 4096 --gather > $O/${T}_mp_c5.json 2> $O/${T}_mp_c5.err &&
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --mode tick > $O/${T}_mp_tick.json 2> $O/${T}_mp_tick.err
