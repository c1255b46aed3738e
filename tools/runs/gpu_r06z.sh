set -o pipefail
cd $GRAFT_REPO_ROOT
# r06z: C3's slice length around r06y's best with the extrapolated key (900 / 950 / 1000 / 1050 /
# 1100, and 1000 again)
O=gpurun_out
T=r06z
L="--companion 0 --reference25 0 --cpu-sample 0 --certify 0 --restatement 1024"
for q in 900 950 1000 1050 1100; do
  timeout -k 10 240 python -u bench.py --config c3 $L --slice $q > $O/${T}_bench_c3_s$q.json 2> $O/${T}_bench_c3_s$q.err || exit 1
done
timeout -k 10 240 python -u bench.py --config c3 $L --slice 1000 > $O/${T}_bench_c3_s1000b.json 2> $O/${T}_bench_c3_s1000b.err
