set -o pipefail
cd $GRAFT_REPO_ROOT
# r06l: the class-order tests (incl. a 2600-instance batch: the order kernel's multi-chunk path),
# then the nested-dissection variant rebuilt on the final source (libmpcq_ndv.so, -DMPCQ_ND: the
# first rows read before the right-hand-side barrier, the spike rows before the post-sweep
# barrier) against the production build on the same box: per iteration, stamps, C3 with parity
O=gpurun_out
T=r06l
timeout -k 10 300 python -u -m pytest tests/test_gpu_order.py -x -v --timeout 240 --timeout-method thread > $O/${T}_pytest_order.log 2>&1 &&
timeout -k 10 240 python -u tools/iterbench.py --N 32 --batches 256 > $O/${T}_iter32_prod.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:ndv timeout -k 10 240 python -u tools/iterbench.py --N 32 --batches 256 > $O/${T}_iter32_ndv.txt 2>&1 &&
timeout -k 10 120 python -u tools/stamps.py --N 32 --batch 256 --copies 0 > $O/${T}_stamps32_prod.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:st32ndv timeout -k 10 120 python -u tools/stamps.py --N 32 --batch 256 --copies 0 --nd > $O/${T}_stamps32_ndv.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:ndv timeout -k 10 240 python -u bench.py --config c3 --steps 5 --warmup 1 --companion 0 --reference25 0 --cpu-sample 0 --certify 0 --restatement 1024 > $O/${T}_bench_c3_ndv.json 2> $O/${T}_bench_c3_ndv.err
