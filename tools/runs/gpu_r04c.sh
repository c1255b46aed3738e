set -o pipefail
cd $GRAFT_REPO_ROOT
# r04c: where the cyclic-reduction iteration spends its time -- per-phase stamps
# (copies of the slowest C2 / C3 instance, alone and co-resident) and factorisation
# cycles, CR vs the round-3 solve
T=r04c
O=gpurun_out
for v in stcr stnocr; do
  f=""; [ $v = stcr ] && f="--cr"
  MPCQ_LIB_VARIANT=exp:$v timeout -k 10 120 python -u tools/stamps.py --N 16 --batch 256 --copies 0 $f > $O/${T}_stamps16_${v}_256.txt 2>&1 || exit 1
  MPCQ_LIB_VARIANT=exp:$v timeout -k 10 120 python -u tools/stamps.py --N 16 --batch 512 --copies 0 $f > $O/${T}_stamps16_${v}_512.txt 2>&1 || exit 1
  MPCQ_LIB_VARIANT=exp:$v timeout -k 10 120 python -u tools/stamps.py --N 32 --batch 256 --copies 19 $f > $O/${T}_stamps32_${v}_256.txt 2>&1 || exit 1
done
for v in ftcr ftnocr; do
  MPCQ_LIB_VARIANT=exp:$v timeout -k 10 120 python -u tools/factime.py 16 > $O/${T}_factime16_${v}.txt 2>&1 || exit 1
  MPCQ_LIB_VARIANT=exp:$v timeout -k 10 120 python -u tools/factime.py 32 > $O/${T}_factime32_${v}.txt 2>&1 || exit 1
done
