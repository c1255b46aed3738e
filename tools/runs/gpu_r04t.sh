set -o pipefail
cd $GRAFT_REPO_ROOT
# r04t: per-horizon latency / batch time on the final build (tools/iterbench.py, C2-shaped batches)
for n in 8 12 16 20 24 28 32 36 40 44 48 49 56 64; do
  timeout -k 10 180 python -u tools/iterbench.py --N $n --reps 2 --batches 256 > gpurun_out/r04t_iter$n.txt 2>&1 || exit 1
done
