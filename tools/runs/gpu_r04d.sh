set -o pipefail
cd $GRAFT_REPO_ROOT
# r04d: the deferred termination check (kDC) -- the GPU suite on it, then same-box A/B
# against the blocking check (exp:nodc) per iteration and on the C2 / C3 launches
T=r04d
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/${T}_pytest_gpu.log 2>&1 &&
timeout -k 10 200 python -u tools/iterbench.py --N 16 > $O/${T}_iter16_dc.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:nodc timeout -k 10 200 python -u tools/iterbench.py --N 16 > $O/${T}_iter16_nodc.txt 2>&1 &&
timeout -k 10 300 python -u tools/iterbench.py --N 32 > $O/${T}_iter32_dc.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:nodc timeout -k 10 300 python -u tools/iterbench.py --N 32 > $O/${T}_iter32_nodc.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --companion 0 --cpu-sample 0 --certify 0 > $O/${T}_bench_c2_dc.json 2> $O/${T}_bench_c2_dc.err &&
MPCQ_LIB_VARIANT=exp:nodc timeout -k 10 300 python -u bench.py --companion 0 --cpu-sample 0 --certify 0 > $O/${T}_bench_c2_nodc.json 2> $O/${T}_bench_c2_nodc.err &&
timeout -k 10 300 python -u bench.py --config c3 --companion 0 --cpu-sample 0 --certify 0 > $O/${T}_bench_c3_dc.json 2> $O/${T}_bench_c3_dc.err &&
MPCQ_LIB_VARIANT=exp:nodc timeout -k 10 300 python -u bench.py --config c3 --companion 0 --cpu-sample 0 --certify 0 > $O/${T}_bench_c3_nodc.json 2> $O/${T}_bench_c3_nodc.err &&
timeout -k 10 300 python -u tools/checkcost.py > $O/${T}_checkcost_dc.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:nodc timeout -k 10 300 python -u tools/checkcost.py > $O/${T}_checkcost_nodc.txt 2>&1
