set -o pipefail
cd $GRAFT_REPO_ROOT
# r06m: sliced solves (mpcq_set_slice) -- the slicing tests (bit-identical outputs against the
# unsliced solve at N = 20 / 32 / 48, polish, class order, warm starts, max_iter, the QP entry
# point; N = 16 compiled out) and the class-order tests, the per-iteration time at N = 32, then C3
# unsliced and at slices of 400 / 800 / 1600 iterations (parity against the restatement on the
# whole batch), then the nested-dissection variant A/B (tools/runs/gpu_r06l.sh's steps)
O=gpurun_out
T=r06m
L="--companion 0 --reference25 0 --cpu-sample 0 --certify 0 --restatement 1024"
timeout -k 10 500 python -u -m pytest tests/test_gpu_slice.py tests/test_gpu_order.py -x -v --timeout 240 --timeout-method thread > $O/${T}_pytest_slice.log 2>&1 &&
timeout -k 10 240 python -u tools/iterbench.py --N 32 --batches 256 > $O/${T}_iter32_prod.txt 2>&1 &&
timeout -k 10 240 python -u bench.py --config c3 $L > $O/${T}_bench_c3_s0.json 2> $O/${T}_bench_c3_s0.err &&
timeout -k 10 240 python -u bench.py --config c3 $L --slice 400 > $O/${T}_bench_c3_s400.json 2> $O/${T}_bench_c3_s400.err &&
timeout -k 10 240 python -u bench.py --config c3 $L --slice 800 > $O/${T}_bench_c3_s800.json 2> $O/${T}_bench_c3_s800.err &&
timeout -k 10 240 python -u bench.py --config c3 $L --slice 1600 > $O/${T}_bench_c3_s1600.json 2> $O/${T}_bench_c3_s1600.err &&
MPCQ_LIB_VARIANT=exp:ndv timeout -k 10 240 python -u tools/iterbench.py --N 32 --batches 256 > $O/${T}_iter32_ndv.txt 2>&1 &&
timeout -k 10 120 python -u tools/stamps.py --N 32 --batch 256 --copies 0 > $O/${T}_stamps32_prod.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:st32ndv timeout -k 10 120 python -u tools/stamps.py --N 32 --batch 256 --copies 0 --nd > $O/${T}_stamps32_ndv.txt 2>&1
