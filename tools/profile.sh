#!/bin/bash
# rocprofv3 evidence for one bench configuration: kernel-trace stats, then the
# HBM counters (FETCH_SIZE and WRITE_SIZE in separate passes, as the gfx950 TCC
# slot budget requires), two SQ passes and the FP64 instruction-count pass.  Counters never share a run with
# --sys-trace / --runtime-trace.  Every GPU step has its own time limit and the
# chain stops at the first failure.
#   bash tools/profile.sh <tag> [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}; shift
ARGS=${@:---config c2}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
# (no companion / reference25 / restatement: the counters would also count their launches of the
# same kernel)
B="python3 $R/bench.py $ARGS --steps 3 --warmup 1 --cpu-sample 0 --certify 0 --companion 0 --reference25 0 --restatement 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B > $OUT/trace.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $B > $OUT/fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $B > $OUT/write.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU \
    --output-format csv -d $OUT/sq -o run -- $B > $OUT/sq.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES \
    --output-format csv -d $OUT/sq2 -o run -- $B > $OUT/sq2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_MFMA_F64 \
    --output-format csv -d $OUT/f64 -o run -- $B > $OUT/f64.log 2>&1
rc=$?
echo "profile rc=$rc" >> $OUT/trace.log
exit $rc
