#!/bin/bash
# GPU box: rocprofv3 kernel trace + PMC passes over config-5 paged batches.
# Usage: bash tools/prof_pages.sh <tag>
set -o pipefail
TAG=${1:-r05}
R=$(pwd)
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 $R/tools/prof_pages.py 100000000 5 > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 1; }
echo trace ok
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU -f csv -d $OUT/pmc1 -o run -- python3 $R/tools/prof_pages.py 100000000 2 > $OUT/pmc1.log 2>&1 || { tail -5 $OUT/pmc1.log; exit 1; }
echo pmc1 ok
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/pmc2 -o run -- python3 $R/tools/prof_pages.py 100000000 2 > $OUT/pmc2.log 2>&1 || { tail -5 $OUT/pmc2.log; exit 1; }
echo pmc2 ok
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/pmc3 -o run -- python3 $R/tools/prof_pages.py 100000000 2 > $OUT/pmc3.log 2>&1 || { tail -5 $OUT/pmc3.log; exit 1; }
echo pmc3 ok
find $OUT -name "*.csv" | head -20
