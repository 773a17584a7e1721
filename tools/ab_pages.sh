# Paged-stream GPU tests, then the config-5 breakdown of the default build (A)
# against abx/libB.so (B), alternating.  Usage: bash tools/ab_pages.sh TAG
set -o pipefail
tag=${1:-ab}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_paged_stream.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
for i in 1 2; do
  timeout -k 10 300 python3 tools/part_breakdown.py 100000000 20 > gpurun_out/${tag}_A$i.txt 2>&1 || { tail -5 gpurun_out/${tag}_A$i.txt; exit 1; }
  grep -E "page_merge|wall" gpurun_out/${tag}_A$i.txt
  ST_LIB=${LIBB:-abx/libB.so} timeout -k 10 300 python3 tools/part_breakdown.py 100000000 20 > gpurun_out/${tag}_B$i.txt 2>&1 || { tail -5 gpurun_out/${tag}_B$i.txt; exit 1; }
  grep -E "page_merge|wall" gpurun_out/${tag}_B$i.txt
done
