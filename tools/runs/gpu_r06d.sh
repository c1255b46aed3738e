set -o pipefail
cd $GRAFT_REPO_ROOT
# r06d: the nested-dissection state solve at N = 32 with one sweep code path (B padded with a
# phantom stage) and no spill in the ADMM loop: C3 against the oracle's restatement, per-iteration
# latency, the N = 32 GPU tests; then the C2 / C5-shard lines of r06b (class order A/B)
O=gpurun_out
timeout -k 10 240 python -u bench.py --config c3 --steps 5 --warmup 1 --companion 0 --reference25 0 --cpu-sample 0 --certify 256 --restatement 1024 > $O/r06d_bench_c3.json 2> $O/r06d_bench_c3.err &&
timeout -k 10 240 python -u tools/iterbench.py --N 32 --batches 256 > $O/r06d_iter32.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_session.py tests/test_gpu_facade.py tests/test_gpu_order.py -x -v -m gpu -k "32 or c3 or C3 or order" --timeout 300 --timeout-method thread > $O/r06d_pytest_n32.log 2>&1 &&
timeout -k 10 300 python -u bench.py --companion 0 --cpu-sample 0 --certify 0 --restatement 256 > $O/r06d_bench_c2.json 2> $O/r06d_bench_c2.err &&
timeout -k 10 300 python -u bench.py --config c5 --batch 4096 --companion 0 --reference25 0 --cpu-sample 0 --certify 0 --restatement 512 > $O/r06d_bench_c5_shard4096.json 2> $O/r06d_bench_c5_shard.err &&
timeout -k 10 300 python -u bench.py --config c5 --batch 4096 --order-by-class 0 --companion 0 --reference25 0 --cpu-sample 0 --certify 0 --restatement 0 > $O/r06d_bench_c5_shard4096_noorder.json 2> $O/r06d_bench_c5_shard_noorder.err &&
# ND at N = 16 (experiment variant libmpcq_nd16.so, -DMPCQ_ND16): per iteration and C2, A/B on this box
timeout -k 10 240 python -u tools/iterbench.py --N 16 --batches 256 512 > $O/r06d_iter16_prod.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:nd16 timeout -k 10 240 python -u tools/iterbench.py --N 16 --batches 256 512 > $O/r06d_iter16_nd16.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:nd16 timeout -k 10 300 python -u bench.py --companion 0 --reference25 0 --cpu-sample 0 --certify 0 --restatement 1024 > $O/r06d_bench_c2_nd16.json 2> $O/r06d_bench_c2_nd16.err
