#!/bin/bash
# PMC passes over tools/microbench/k1_explore (diagnostic).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_explore; mkdir -p $O
timeout -k 10 120 ./tools/microbench/k1_explore > $O/plain.txt 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES -f csv -d $O/sq -o run -- ./tools/microbench/k1_explore > $O/sq.txt 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum FETCH_SIZE GRBM_GUI_ACTIVE -f csv -d $O/ta -o run -- ./tools/microbench/k1_explore > $O/ta.txt 2>&1 || exit 1
echo pmc done
