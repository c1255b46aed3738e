set -o pipefail
cd $GRAFT_REPO_ROOT
# r04h: stamps of wave 0 and of the last wave (the rhs phase split from its barrier wait)
for v in st0 stL; do
  for n in 16 48 64; do
    MPCQ_LIB_VARIANT=exp:$v timeout -k 10 120 python -u tools/stamps.py --N $n --batch 256 > gpurun_out/r04h_stamps${n}_$v.txt 2>&1 || exit 1
  done
done
