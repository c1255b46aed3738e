set -o pipefail
cd $GRAFT_REPO_ROOT
# r04f: the round's build -- GPU suite, smoke, every bench line, the rocprof passes
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04f_pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04f_smoke.log 2>&1 &&
bash tools/bench_all.sh r04f &&
for n in 16 32 48 64; do
  timeout -k 10 120 python -u tools/stamps.py --N $n --batch 256 > gpurun_out/r04f_stamps$n.txt 2>&1 || exit 1
done
