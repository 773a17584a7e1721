#!/bin/bash
# PMC passes (one group per run) on the rehash kernels of a short bench.
R=$(pwd); TAG=${1:-k1}; RX=${2:-segment_hash|level16|upper16}
export TMPDIR=/tmp
SHORT="$R/bench.py --steps 5 --warmup 1 --no-cpu --no-extras --no-pmc"
i=0
for G in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "MeanOccupancyPerCU" \
         "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum" \
         "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $G --kernel-include-regex "$RX" -f csv -d $R/gpurun_out/pmc_$TAG/p$i -o run -- python3 $SHORT > /dev/null 2> $R/gpurun_out/pmc_$TAG/p$i.err || { echo "pass $i failed"; exit 1; }
done
