set -o pipefail
cd $GRAFT_REPO_ROOT
# r06c: the nested-dissection state solve at N = 32 (kND): C3 against the oracle's restatement
# (statuses / iterations on all 1024 instances), per-iteration latency, the N = 32 GPU tests
O=gpurun_out
timeout -k 10 240 python -u bench.py --config c3 --steps 5 --warmup 1 --companion 0 --reference25 0 --cpu-sample 0 --certify 256 --restatement 1024 > $O/r06c_bench_c3.json 2> $O/r06c_bench_c3.err &&
timeout -k 10 240 python -u tools/iterbench.py --N 32 --batches 256 > $O/r06c_iter32.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_session.py tests/test_gpu_facade.py -x -v -m gpu -k "32 or c3 or C3" --timeout 300 --timeout-method thread > $O/r06c_pytest_n32.log 2>&1
