#!/bin/bash
# One GPU session: parity tests, smoke, benches, rocprofv3 kernel-trace stats.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-r01}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -m pytest tests -x -q -m gpu > $OUT/pytest_gpu_$TAG.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 &&
timeout -k 10 600 python bench.py > $OUT/bench_c2_$TAG.json 2> $OUT/bench_c2_$TAG.err &&
timeout -k 10 600 python bench.py --config c3 --cpu-sample 256 > $OUT/bench_c3_$TAG.json 2> $OUT/bench_c3_$TAG.err &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o c2 -- python3 $R/bench.py --steps 5 --warmup 1 --cpu-sample 0 > $OUT/prof_$TAG.log 2>&1
echo "EXIT $?" >> $OUT/pytest_gpu_$TAG.log
