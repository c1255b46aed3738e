set -o pipefail
cd $GRAFT_REPO_ROOT
# r04e: where the GPU's solution leaves the oracle's per horizon, and
# the per-iteration time beyond 48 stages against the number of instances in flight
# (the per-instance share of each XCD's L2), and the C3 LDS bank-conflict experiment (lanes 12..15 of the sweep broadcasting lanes 0..3
# at N = 32 too): per-iteration time and the LDS counters, production vs exp:rr12
T=r04e
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 400 python -u tools/drift.py --horizons 16 32 48 49 50 57 64 > $O/${T}_drift.txt 2>&1 &&
for n in 48 49 64; do timeout -k 10 300 python -u tools/iterbench.py --N $n --reps 3 --batches 32 64 128 256 > $O/${T}_occ_n$n.txt 2>&1 || exit 1; done &&
timeout -k 10 300 python -u tools/iterbench.py --N 32 > $O/${T}_iter32_prod.txt 2>&1 &&
MPCQ_LIB_VARIANT=exp:rr12 timeout -k 10 300 python -u tools/iterbench.py --N 32 > $O/${T}_iter32_rr12.txt 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
B="python3 $GRAFT_REPO_ROOT/bench.py --config c3 --steps 3 --warmup 1 --cpu-sample 0 --certify 0 --companion 0 --restatement 0" &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS --output-format csv -d $O/prof_${T}_lds_prod -o run -- $B > $O/${T}_lds_prod.log 2>&1 &&
export MPCQ_LIB_VARIANT=exp:rr12 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS --output-format csv -d $O/prof_${T}_lds_rr12 -o run -- $B > $O/${T}_lds_rr12.log 2>&1
