set -o pipefail
cd $GRAFT_REPO_ROOT
# r06ac: the 2-rank gloo rehearsal of the launcher on C3 (each rank slices its own 1024 instances)
O=gpurun_out
T=r06ac
MPCQ_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --config c3 --companion 0 --reference25 0 --cpu-sample 0 --certify 0 > $O/${T}_rehearsal_2rank_c3.json 2> $O/${T}_rehearsal_2rank_c3.err
