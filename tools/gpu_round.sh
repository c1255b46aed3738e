#!/bin/bash
# One GPU session of a round: the -m gpu suite, smoke, the C2 / C3 bench lines
# (headline + companion mode) and a rocprofv3 kernel-trace of the C2 headline.
# Every GPU step has its own time limit; the chain stops at the first failure.
#   bash tools/gpu_round.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:?tag}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/${TAG}_pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${TAG}_smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $OUT/${TAG}_bench_c2.json 2> $OUT/${TAG}_bench_c2.err &&
timeout -k 10 300 python -u bench.py --config c3 > $OUT/${TAG}_bench_c3.json 2> $OUT/${TAG}_bench_c3.err &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_prof -o c2 -- python3 $R/bench.py --steps 5 --warmup 1 --cpu-sample 0 --certify 0 --companion 0 > $OUT/${TAG}_prof.log 2>&1
rc=$?
echo "rc=$rc" >> $OUT/${TAG}_pytest_gpu.log
exit $rc
