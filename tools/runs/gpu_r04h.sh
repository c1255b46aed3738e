set -o pipefail
cd $GRAFT_REPO_ROOT
# r04h: stamps of wave 0 and of the last wave (the rhs phase split from its barrier wait)
for v in st0 stL; do
  for n in 16 48 64; do
    MPCQ_LIB_VARIANT=exp:$v timeout -k 10 120 python -u tools/stamps.py --N $n --batch 256 > gpurun_out/r04h_stamps${n}_$v.txt 2>&1 || exit 1
  done
done
# the lag-style outward sweep beyond 32 stages (variant lagout: horizons 33 40 48 49 56 64)
MPCQ_LIB_VARIANT=exp:lagout timeout -k 10 600 python -u -m pytest tests/test_gpu_horizons.py -x -v -m gpu --timeout 300 --timeout-method thread -k "horizon_parity and (33 or 40 or 48 or 49 or 64)" > gpurun_out/r04h_pytest_lagout.log 2>&1 &&
for n in 40 48 56 64; do
  MPCQ_LIB_VARIANT=exp:lagout timeout -k 10 180 python -u tools/iterbench.py --N $n --reps 2 --batches 32 256 > gpurun_out/r04h_iter${n}_lagout.txt 2>&1 || exit 1
done
# (zyc: lagout + z / y / x in private memory + the rhs operands in two batches, N > 48)
MPCQ_LIB_VARIANT=exp:zyc timeout -k 10 600 python -u -m pytest tests/test_gpu_horizons.py -x -v -m gpu --timeout 300 --timeout-method thread -k "horizon_parity and (49 or 64)" > gpurun_out/r04h_pytest_zyc.log 2>&1 &&
for n in 56 64; do
  MPCQ_LIB_VARIANT=exp:zyc timeout -k 10 180 python -u tools/iterbench.py --N $n --reps 2 --batches 32 256 > gpurun_out/r04h_iter${n}_zyc.txt 2>&1 || exit 1
done
