set -o pipefail
cd $GRAFT_REPO_ROOT
# r06y: the resumed launch ordered by the iterations left, extrapolated from the primal / dual
# residuals' decay over the second half of the slice (Spearman +0.995 at Q = 1200 offline) --
# the slicing tests, then C3 at slices of 600 / 800 / 1000 / 1200
O=gpurun_out
T=r06y
L="--companion 0 --reference25 0 --cpu-sample 0 --certify 0 --restatement 1024"
timeout -k 10 400 python -u -m pytest tests/test_gpu_slice.py -x -v --timeout 240 --timeout-method thread > $O/${T}_pytest_slice.log 2>&1 || exit 1
for q in 600 800 1000 1200; do
  timeout -k 10 240 python -u bench.py --config c3 $L --slice $q > $O/${T}_bench_c3_s$q.json 2> $O/${T}_bench_c3_s$q.err || exit 1
done
