set -o pipefail
cd $GRAFT_REPO_ROOT
# r05c: the explicit inverse with the product's loads pipelined: smoke, per-iteration latency, C2
O=gpurun_out
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/r05c_smoke.log 2>&1 &&
timeout -k 10 300 python -u tools/iterbench.py --N 16 --reps 3 > $O/r05c_iter16.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --restatement 1024 --certify 0 --cpu-sample 0 > $O/r05c_bench_c2.json 2> $O/r05c_bench_c2.err
