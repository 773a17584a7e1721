# Config-5 breakdowns of the in-tree build and of each abx/lib<V>.so named on
# the command line.  Every variant must compute the same results: a variant
# that skips work leaves offsets the next batch indexes (a GPU fault).  No
# tests run here.  Usage: bash tools/ab_variants.sh TAG V1 V2 ...
set -o pipefail
tag=${1:-abv}; shift
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/part_breakdown.py 100000000 20 > gpurun_out/${tag}_base.txt 2>&1 || { tail -5 gpurun_out/${tag}_base.txt; exit 1; }
echo base; grep -E "page_merge|wall" gpurun_out/${tag}_base.txt
for v in "$@"; do
  ST_LIB=abx/lib$v.so timeout -k 10 300 python3 tools/part_breakdown.py 100000000 20 > gpurun_out/${tag}_$v.txt 2>&1 || { tail -5 gpurun_out/${tag}_$v.txt; exit 1; }
  echo $v; grep -E "page_merge|wall" gpurun_out/${tag}_$v.txt
done
