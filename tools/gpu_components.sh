#!/bin/bash
# Benches and rocprofv3 evidence of the planner and closed-loop session paths.
#   bash tools/gpu_components.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-r01}
mkdir -p $OUT
cd $R
timeout -k 10 300 python bench.py --mode plan --cpu-sample 4096 > $OUT/bench_plan_$TAG.json 2> $OUT/bench_plan_$TAG.err &&
timeout -k 10 300 python bench.py --mode tick --steps 20 --warmup 4 > $OUT/bench_tick_c2_$TAG.json 2> $OUT/bench_tick_c2_$TAG.err &&
timeout -k 10 300 python bench.py --mode tick --config c5 --batch 32768 --steps 5 --warmup 2 --cpu-sample 0 > $OUT/bench_tick_c5_$TAG.json 2> $OUT/bench_tick_c5_$TAG.err &&
bash tools/profile.sh ${TAG}_plan --mode plan &&
bash tools/profile.sh ${TAG}_tick --mode tick
