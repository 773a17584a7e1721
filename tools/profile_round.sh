#!/bin/bash
# Profile bench.py on the GPU box: kernel-trace stats of the bench command and
# separate PMC passes (one counter group per run, as the pool requires).
# Usage (on the box, from the repo root): bash tools/profile_round.sh <tag>
set -euo pipefail
TAG=${1:-r1}
R=$(pwd)
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="$R/bench.py --steps 20 --warmup 5"
SHORT="$R/bench.py --steps 5 --warmup 1 --no-cpu --no-extras"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 $BENCH > $OUT/bench_trace.json 2> $OUT/bench_trace.err
echo "trace done"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/pmc_fetch -o run -- python3 $SHORT > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err
echo "fetch done"
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/pmc_write -o run -- python3 $SHORT > $OUT/pmc_write.json 2> $OUT/pmc_write.err
echo "write done"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -f csv -d $OUT/pmc_sq -o run -- python3 $SHORT > $OUT/pmc_sq.json 2> $OUT/pmc_sq.err
echo "sq done"
