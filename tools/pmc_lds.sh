#!/bin/bash
# LDS / issue counters of the engine kernel at one instance per CU (batch 256) and two (512).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_lds
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for B in 256 512; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU \
    --output-format csv -d $OUT/b$B -o run -- python3 $R/bench.py --batch $B --steps 2 --warmup 1 --cpu-sample 0 > $OUT/b$B.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU \
    --output-format csv -d $OUT/b${B}s -o run -- python3 $R/bench.py --batch $B --steps 2 --warmup 1 --cpu-sample 0 > $OUT/b${B}s.log 2>&1 || exit 1
done
