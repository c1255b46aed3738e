set -o pipefail
cd $GRAFT_REPO_ROOT
# r05e: explicit inverse, r by row broadcast, rebalanced split: smoke, latency, stamps, C2
O=gpurun_out
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/r05e_smoke.log 2>&1 &&
timeout -k 10 300 python -u tools/iterbench.py --N 16 --reps 3 --batches 256 > $O/r05e_iter16.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:kist0 timeout -k 10 120 python -u tools/stamps.py --ki --copies 0 --batch 256 > $O/r05e_stamps_w0.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --restatement 1024 --certify 0 --cpu-sample 0 --companion 0 > $O/r05e_bench_c2.json 2> $O/r05e_bench_c2.err
