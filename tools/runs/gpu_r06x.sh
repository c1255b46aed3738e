set -o pipefail
cd $GRAFT_REPO_ROOT
# r06x: the C3 line again after r06w's profile was summarised per solve (prof_summary counted
# r06w's two equally sized launches per sliced solve as two solves on the box), so that it
# quotes the per-solve traffic; the default line (C2) beside it
O=gpurun_out
T=r06x
timeout -k 10 300 python -u bench.py --config c3 > $O/${T}_bench_c3.json 2> $O/${T}_bench_c3.err &&
timeout -k 10 300 python -u bench.py > $O/${T}_bench_c2.json 2> $O/${T}_bench_c2.err
