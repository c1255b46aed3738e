set -o pipefail
cd $GRAFT_REPO_ROOT
# r06e: the nested-dissection solve at N = 32 with the separator's right-hand side from its own
# slot: C3 vs the oracle's restatement, per-iteration latency, per-phase stamps (ND vs the round-5
# sweep, same box), the N = 32 / order GPU tests; ND at N = 16 (variant) A/B; C2 and C5-shard lines
O=gpurun_out
timeout -k 10 240 python -u bench.py --config c3 --steps 5 --warmup 1 --companion 0 --reference25 0 --cpu-sample 0 --certify 256 --restatement 1024 > $O/r06e_bench_c3.json 2> $O/r06e_bench_c3.err &&
timeout -k 10 240 python -u tools/iterbench.py --N 32 --batches 256 > $O/r06e_iter32.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:st32nd timeout -k 10 120 python -u tools/stamps.py --N 32 --batch 256 --copies 0 --nd > $O/r06e_stamps32_nd.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:st32old timeout -k 10 120 python -u tools/stamps.py --N 32 --batch 256 --copies 0 > $O/r06e_stamps32_old.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_session.py tests/test_gpu_facade.py tests/test_gpu_order.py -x -v -m gpu -k "32 or c3 or C3 or order" --timeout 300 --timeout-method thread > $O/r06e_pytest_n32.log 2>&1 &&
timeout -k 10 240 python -u tools/iterbench.py --N 16 --batches 256 512 > $O/r06e_iter16_prod.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:nd16 timeout -k 10 240 python -u tools/iterbench.py --N 16 --batches 256 512 > $O/r06e_iter16_nd16.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --companion 0 --cpu-sample 0 --certify 0 --restatement 256 > $O/r06e_bench_c2.json 2> $O/r06e_bench_c2.err &&
MPCQ_LIB_VARIANT=exp:nd16 timeout -k 10 300 python -u bench.py --companion 0 --reference25 0 --cpu-sample 0 --certify 0 --restatement 1024 > $O/r06e_bench_c2_nd16.json 2> $O/r06e_bench_c2_nd16.err &&
timeout -k 10 300 python -u bench.py --config c5 --batch 4096 --companion 0 --reference25 0 --cpu-sample 0 --certify 0 --restatement 512 > $O/r06e_bench_c5_shard4096.json 2> $O/r06e_bench_c5_shard.err &&
timeout -k 10 300 python -u bench.py --config c5 --batch 4096 --order-by-class 0 --companion 0 --reference25 0 --cpu-sample 0 --certify 0 --restatement 0 > $O/r06e_bench_c5_shard4096_noorder.json 2> $O/r06e_bench_c5_shard_noorder.err
