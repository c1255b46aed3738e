set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
# r03s: per-phase cycles alone (256 copies) vs co-resident (512 copies), N = 16 and 32
for n in 16; do
  for b in 256 512; do
    timeout -k 10 300 env MPCQ_LIB_VARIANT=stamps python -u tools/stamps.py --N $n --copies 0 --batch $b > $O/r03s_stamps${n}_b$b.txt 2>&1 || exit 1
  done
done
