# GPU box: PMC passes (FETCH_SIZE, WRITE_SIZE, SQ waits) over config-5 paged batches; per-kernel
# values of the last paged batch.  Usage: bash tools/r06_pmc5.sh TAG
set -o pipefail
TAG=${1:-x}
R=$(pwd)
OUT=$R/gpurun_out/pmc5_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/p_fetch -o run -- python3 $R/tools/prof_pages.py 100000000 3 > $OUT/fetch.log 2>&1 || { tail -5 $OUT/fetch.log; exit 1; }
echo fetch ok
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/p_write -o run -- python3 $R/tools/prof_pages.py 100000000 3 > $OUT/write.log 2>&1 || { tail -5 $OUT/write.log; exit 1; }
echo write ok
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES -f csv -d $OUT/p_sq -o run -- python3 $R/tools/prof_pages.py 100000000 3 > $OUT/sq.log 2>&1 || { tail -5 $OUT/sq.log; exit 1; }
echo sq ok
python3 $R/tools/pmc_last.py $OUT > $OUT/summary.txt && cat $OUT/summary.txt
