set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
timeout -k 10 240 python -u bench.py > $O/r02j_bench_c2.json 2> $O/r02j_bench_c2.err &&
timeout -k 10 240 python -u bench.py --no-polish > $O/r02j_bench_c2_nopolish.json 2> $O/r02j_bench_c2_nopolish.err &&
timeout -k 10 240 python -u bench.py --config c3 > $O/r02j_bench_c3.json 2> $O/r02j_bench_c3.err &&
timeout -k 10 240 python -u bench.py --config c1 > $O/r02j_bench_c1.json 2> $O/r02j_bench_c1.err &&
timeout -k 10 300 python -u bench.py --config c4 --steps 3 --warmup 1 > $O/r02j_bench_c4_1gpu.json 2> $O/r02j_bench_c4.err &&
timeout -k 10 300 python -u bench.py --config c5 --steps 3 --warmup 1 > $O/r02j_bench_c5_1gpu.json 2> $O/r02j_bench_c5.err &&
bash tools/profile.sh r02j
