set -o pipefail
cd $GRAFT_REPO_ROOT
# r06ab: the round's final build (r06aa with the header comment on the key corrected: a new stamp) (sliced solves beyond 16 stages, resumed once by the extrapolated iterations left, the resumed launch sized on the device; bench.py slicing C3 at 1000 by
# default) -- smoke, the whole GPU suite, per-iteration times, then every configuration profiled
# (tools/profile.sh, summarised on the box into profiles/pmc_traffic.json) before its bench line:
# C2, C3 (sliced: figures per solve), the C4 / C5 rank shards, whole C4 / C5 on one GPU; C1, the
# session tick, the planner, the 2-rank gloo rehearsal
O=gpurun_out
T=r06ab
prof() {  # tag key instances bench-args...
  local tag=$1 key=$2 n=$3; shift 3
  bash tools/profile.sh $tag "$@" && python3 tools/prof_summary.py $tag --key $key --instances $n > $O/${tag}_summary.txt 2>&1
}
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/${T}_pytest_gpu.log 2>&1 &&
timeout -k 10 240 python -u tools/iterbench.py --N 16 --batches 256 > $O/${T}_iter16.txt 2>&1 &&
timeout -k 10 240 python -u tools/iterbench.py --N 32 --batches 256 > $O/${T}_iter32.txt 2>&1 &&
prof ${T} c2_N16_B1024 1024 --config c2 &&
prof ${T}c3 c3_N32_B1024_s1000 1024 --config c3 &&
prof ${T}c4s c4_N16_B8192 8192 --config c4 --batch 8192 &&
prof ${T}c5s c5_N16_B4096 4096 --config c5 --batch 4096 &&
timeout -k 10 300 python -u bench.py > $O/${T}_bench_c2.json 2> $O/${T}_bench_c2.err &&
timeout -k 10 300 python -u bench.py --config c3 > $O/${T}_bench_c3.json 2> $O/${T}_bench_c3.err &&
timeout -k 10 300 python -u bench.py --config c4 --batch 8192 --companion 0 --reference25 0 --cpu-sample 0 --certify 0 --restatement 512 > $O/${T}_bench_c4_shard8192.json 2> $O/${T}_bench_c4_shard.err &&
timeout -k 10 300 python -u bench.py --config c5 --batch 4096 --companion 0 --reference25 0 --cpu-sample 0 --certify 0 --restatement 512 > $O/${T}_bench_c5_shard4096.json 2> $O/${T}_bench_c5_shard.err &&
mkdir -p $O/profiles_${T} && cp profiles/${T}*_summary.md profiles/${T}*_kernel_stats.csv profiles/pmc_traffic.json $O/profiles_${T}/ &&
prof ${T}c5 c5_N16_B32768 32768 --config c5 &&
prof ${T}c4 c4_N16_B65536 65536 --config c4 &&
timeout -k 10 300 python -u bench.py --config c5 --steps 3 --warmup 1 > $O/${T}_bench_c5_1gpu.json 2> $O/${T}_bench_c5.err &&
timeout -k 10 300 python -u bench.py --config c4 --steps 3 --warmup 1 > $O/${T}_bench_c4_1gpu.json 2> $O/${T}_bench_c4.err &&
timeout -k 10 240 python -u bench.py --config c1 > $O/${T}_bench_c1.json 2> $O/${T}_bench_c1.err &&
timeout -k 10 300 python -u bench.py --mode tick --steps 20 --warmup 4 > $O/${T}_bench_tick_c2.json 2> $O/${T}_bench_tick_c2.err &&
timeout -k 10 300 python -u bench.py --mode plan --cpu-sample 4096 > $O/${T}_bench_plan.json 2> $O/${T}_bench_plan.err &&
MPCQ_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --companion 0 --reference25 0 --cpu-sample 0 --certify 0 > $O/${T}_rehearsal_2rank_self.json 2> $O/${T}_rehearsal_2rank_self.err &&
cp profiles/${T}*_summary.md profiles/${T}*_kernel_stats.csv profiles/pmc_traffic.json $O/profiles_${T}/
