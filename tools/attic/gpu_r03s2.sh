set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
# r03s2: the split sweep (round-3 form: select rotation, laundered ids) at N = 16 / 32
# against the lagging sweep of the production build; same box
timeout -k 10 300 python -u tools/iterbench.py --reps 3 > $O/r03s2_iter16_lag.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:split16 timeout -k 10 300 python -u tools/iterbench.py --reps 3 > $O/r03s2_iter16_split.txt 2>&1 &&
timeout -k 10 300 python -u tools/iterbench.py --N 32 --reps 2 > $O/r03s2_iter32_lag.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:split32 timeout -k 10 300 python -u tools/iterbench.py --N 32 --reps 2 > $O/r03s2_iter32_split.txt 2>&1
