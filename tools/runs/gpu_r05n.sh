set -o pipefail
cd $GRAFT_REPO_ROOT
# r05n: round-5 final build (lazy Gauss-Jordan pivot rows): every bench line of DESIGN §5
# and the stamped rocprof passes for C2 and C3
O=gpurun_out
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/r05n_smoke.log 2>&1 &&
bash tools/bench_all.sh r05n
