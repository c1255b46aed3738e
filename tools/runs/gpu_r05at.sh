set -o pipefail
cd $GRAFT_REPO_ROOT
# r05at: round-5 final build (nop-elision pass, max-ilp at every horizon but 40): smoke, every
# bench line of DESIGN §5 and the stamped rocprof passes for C2 and C3 (part 1; part 2 =
# gpu_r05au.sh: GPU suite, per-iteration at N = 16..64)
O=gpurun_out
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/r05at_smoke.log 2>&1 &&
bash tools/bench_all.sh r05at
