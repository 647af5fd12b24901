#!/bin/bash
# SQ counter passes over tools/diag/bwd_once.py (run via gpurun from the repo root).
#   tools/diag/pmc_bwd.sh [TAG [SIZE B]]   (default: pmc_bwd, config 3's 128 64)
set -e
ROOT=$(pwd)
TAG=${1:-pmc_bwd}
ARGS="${2:-128} ${3:-64}"
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS" \
           "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INSTS_SALU" \
           "SQ_INSTS_VALU_FMA_F64 SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o p$i -- python3 $ROOT/tools/diag/bwd_once.py $ARGS > $OUT/p$i.log 2>&1
done
find $OUT -name "*counter_collection.csv"
