#!/bin/bash
# Bench matrix on one GPU: the default headline (polish) with its CPU baseline and
# certificate, then polish off and the adaptive-rho interval variants (no CPU leg).
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-m}
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u bench.py > $OUT/bench_c2_pol_$TAG.json 2> $OUT/bench_c2_pol_$TAG.err &&
timeout -k 10 200 python -u bench.py --no-polish --cpu-sample 0 > $OUT/bench_c2_nopol_$TAG.json 2> $OUT/bench_c2_nopol_$TAG.err &&
timeout -k 10 200 python -u bench.py --rho-interval 25 --cpu-sample 0 > $OUT/bench_c2_pol25_$TAG.json 2> $OUT/bench_c2_pol25_$TAG.err &&
timeout -k 10 200 python -u bench.py --no-polish --rho-interval 25 --cpu-sample 0 > $OUT/bench_c2_nopol25_$TAG.json 2> $OUT/bench_c2_nopol25_$TAG.err &&
timeout -k 10 300 python -u bench.py --config c3 --cpu-sample 0 --certify 256 > $OUT/bench_c3_pol_$TAG.json 2> $OUT/bench_c3_pol_$TAG.err &&
timeout -k 10 300 python -u bench.py --config c3 --rho-interval 25 --cpu-sample 0 --certify 256 > $OUT/bench_c3_pol25_$TAG.json 2> $OUT/bench_c3_pol25_$TAG.err
echo "rc=$?" > $OUT/modes_$TAG.rc
