set -o pipefail
cd $GRAFT_REPO_ROOT
# r06h (3 of 3): the whole-batch C4 / C5 on one GPU (profiled, then their lines), C1, the session
# tick, the planner, and the 2-rank gloo rehearsal of the launcher -- same build as r06g (its
# profiles/pmc_traffic.json committed before this call)
O=gpurun_out
T=${T:-r06h}
prof() {
  local tag=$1 key=$2 n=$3; shift 3
  bash tools/profile.sh $tag "$@" && python3 tools/prof_summary.py $tag --key $key --instances $n > $O/${tag}_summary.txt 2>&1
}
prof ${T}c5 c5_N16_B32768 32768 --config c5 &&
prof ${T}c4 c4_N16_B65536 65536 --config c4 &&
timeout -k 10 300 python -u bench.py --config c5 --steps 3 --warmup 1 > $O/${T}_bench_c5_1gpu.json 2> $O/${T}_bench_c5.err &&
timeout -k 10 300 python -u bench.py --config c4 --steps 3 --warmup 1 > $O/${T}_bench_c4_1gpu.json 2> $O/${T}_bench_c4.err &&
timeout -k 10 240 python -u bench.py --config c1 > $O/${T}_bench_c1.json 2> $O/${T}_bench_c1.err &&
timeout -k 10 300 python -u bench.py --mode tick --steps 20 --warmup 4 > $O/${T}_bench_tick_c2.json 2> $O/${T}_bench_tick_c2.err &&
timeout -k 10 300 python -u bench.py --mode plan --cpu-sample 4096 > $O/${T}_bench_plan.json 2> $O/${T}_bench_plan.err &&
MPCQ_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --companion 0 --reference25 0 --cpu-sample 0 --certify 0 > $O/${T}_rehearsal_2rank_self.json 2> $O/${T}_rehearsal_2rank_self.err &&
mkdir -p $O/profiles_${T} && cp profiles/${T}*_summary.md profiles/${T}*_kernel_stats.csv profiles/pmc_traffic.json $O/profiles_${T}/
