set -o pipefail
cd $GRAFT_REPO_ROOT
# r06i: the nested-dissection variant with the first rows read before the right-hand-side barrier
# and the spike rows before the post-sweep barrier (libmpcq_ndv.so, -DMPCQ_ND): per iteration and
# stamps against the production build on the same box
O=gpurun_out
timeout -k 10 240 python -u tools/iterbench.py --N 32 --batches 256 > $O/r06i_iter32_prod.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:ndv timeout -k 10 240 python -u tools/iterbench.py --N 32 --batches 256 > $O/r06i_iter32_ndv.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:st32ndv timeout -k 10 120 python -u tools/stamps.py --N 32 --batch 256 --copies 0 --nd > $O/r06i_stamps32_ndv.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:ndv timeout -k 10 240 python -u bench.py --config c3 --steps 5 --warmup 1 --companion 0 --reference25 0 --cpu-sample 0 --certify 0 --restatement 1024 > $O/r06i_bench_c3_ndv.json 2> $O/r06i_bench_c3_ndv.err
