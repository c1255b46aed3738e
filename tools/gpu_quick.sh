#!/bin/bash
# Quick GPU check: parity tests, stamps breakdown, default bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-q}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -s -m gpu > $OUT/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/stamps.py > $OUT/stamps_$TAG.log 2>&1 &&
timeout -k 10 300 python tools/stamps.py --batch 256 >> $OUT/stamps_$TAG.log 2>&1 &&
timeout -k 10 600 python bench.py --cpu-sample 256 > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err &&
timeout -k 10 300 python tools/iterbench.py > $OUT/iter_$TAG.txt 2>&1
