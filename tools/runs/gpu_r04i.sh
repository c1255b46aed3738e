set -o pipefail
cd $GRAFT_REPO_ROOT
# r04i: lane-interleaved loop coefficients beyond 49 stages + the lag-style outward sweep
# at 33..48 stages -- GPU suite, per-iteration latency beyond 32 stages
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04i_pytest_gpu.log 2>&1 &&
for n in 40 48 50 56 64; do
  timeout -k 10 180 python -u tools/iterbench.py --N $n --reps 2 --batches 32 256 > gpurun_out/r04i_iter$n.txt 2>&1 || exit 1
done
# same-box control: the CSC gathers (-DMPCQ_NO_OPBLK)
for n in 50 64; do
  MPCQ_LIB_VARIANT=exp:noop timeout -k 10 180 python -u tools/iterbench.py --N $n --reps 2 --batches 32 256 > gpurun_out/r04i_iter${n}_noop.txt 2>&1 || exit 1
done
