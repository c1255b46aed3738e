set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
# r03n: A/B beyond 32 stages: production (F row in the workspace + z constants in private memory) vs F held vs both held
for v in prod frheld bothheld; do
  if [ $v = prod ]; then E=""; else E="MPCQ_LIB_VARIANT=exp:$v"; fi
  for n in 48 64; do
    timeout -k 10 300 env $E python -u tools/iterbench.py --N $n --reps 2 > $O/r03n_${v}_iter$n.txt 2>&1 || exit 1
  done
done
