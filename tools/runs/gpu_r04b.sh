set -o pipefail
cd $GRAFT_REPO_ROOT
# r04b: the cyclic-reduction solve (kCR, N % 4 == 0, 8..32) -- targeted parity at the
# CR horizons, then same-box A/B against the round-3 solve (exp:nocr) per iteration
# and on the C2 / C3 launches
T=r04b
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_horizons.py -x -v -m gpu --timeout 200 --timeout-method thread -k "qp_solve_vs_oracle or fused_vs_oracle or admm_c2_full or headline_c2 or polish_reaches or horizon_parity and (8 or 12 or 20 or 24 or 28)" > $O/${T}_pytest_cr.log 2>&1 &&
timeout -k 10 200 python -u tools/iterbench.py --N 16 > $O/${T}_iter16_cr.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:nocr timeout -k 10 200 python -u tools/iterbench.py --N 16 > $O/${T}_iter16_nocr.txt 2>&1 &&
timeout -k 10 300 python -u tools/iterbench.py --N 32 > $O/${T}_iter32_cr.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:nocr timeout -k 10 300 python -u tools/iterbench.py --N 32 > $O/${T}_iter32_nocr.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --companion 0 --cpu-sample 0 --certify 0 > $O/${T}_bench_c2_cr.json 2> $O/${T}_bench_c2_cr.err &&
MPCQ_LIB_VARIANT=exp:nocr timeout -k 10 300 python -u bench.py --companion 0 --cpu-sample 0 --certify 0 > $O/${T}_bench_c2_nocr.json 2> $O/${T}_bench_c2_nocr.err &&
timeout -k 10 300 python -u bench.py --config c3 --companion 0 --cpu-sample 0 --certify 0 > $O/${T}_bench_c3_cr.json 2> $O/${T}_bench_c3_cr.err &&
MPCQ_LIB_VARIANT=exp:nocr timeout -k 10 300 python -u bench.py --config c3 --companion 0 --cpu-sample 0 --certify 0 > $O/${T}_bench_c3_nocr.json 2> $O/${T}_bench_c3_nocr.err
