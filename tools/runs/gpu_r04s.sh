set -o pipefail
cd $GRAFT_REPO_ROOT
# r04s: the self-launching bench at 4 ranks sharing the box's GPU (gloo rehearsal of the N > 1 path)
MPCQ_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 4 --companion 0 --cpu-sample 0 --certify 0 > gpurun_out/r04s_rehearsal_4rank_self.json 2> gpurun_out/r04s_rehearsal_4rank_self.err &&
MPCQ_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 4 --config c4 --steps 3 --warmup 1 --companion 0 --cpu-sample 0 --certify 0 --restatement 256 > gpurun_out/r04s_rehearsal_4rank_c4.json 2> gpurun_out/r04s_rehearsal_4rank_c4.err
