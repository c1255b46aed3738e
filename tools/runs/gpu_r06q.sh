set -o pipefail
cd $GRAFT_REPO_ROOT
# r06q: resumed slices ordered by the primal residual over its tolerance at suspension (the
# farthest from convergence first) -- the slicing tests (incl. a 2100-instance compaction), then
# C3 at slices of 800 / 1200 / 1600 / 2000 (parity against the restatement on the whole batch)
O=gpurun_out
T=r06q
L="--companion 0 --reference25 0 --cpu-sample 0 --certify 0 --restatement 1024"
timeout -k 10 400 python -u -m pytest tests/test_gpu_slice.py -x -v --timeout 240 --timeout-method thread > $O/${T}_pytest_slice.log 2>&1 || exit 1
for q in 800 1200 1600 2000; do
  timeout -k 10 240 python -u bench.py --config c3 $L --slice $q > $O/${T}_bench_c3_s$q.json 2> $O/${T}_bench_c3_s$q.err || exit 1
done
