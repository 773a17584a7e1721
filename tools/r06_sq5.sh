# GPU box: one SQ-counter pass (wave cycles by state) over config-5 paged batches; per-kernel values of the last
# batch.  Usage: bash tools/r06_sq5.sh TAG
set -o pipefail
TAG=${1:-x}
R=$(pwd)
OUT=$R/gpurun_out/sq5_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU -f csv -d $OUT/p_sq -o run -- python3 $R/tools/prof_pages.py 100000000 3 > $OUT/sq.log 2>&1 || { tail -5 $OUT/sq.log; exit 1; }
python3 $R/tools/pmc_last.py $OUT > $OUT/summary.txt && grep -E "kernel|k_verify_cap|k_segment_hash_perm|k_page_merge|k_merge_keys|k_run_plan" $OUT/summary.txt
