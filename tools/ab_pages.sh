# Paged-stream + term-key/leveldb GPU tests, then the config-5 breakdown of the
# default build (A) against abx/libB.so (B).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_paged_stream.py tests/test_term_keys.py tests/test_leveldb_format.py \
    -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05i_tests.log 2>&1 || { tail -30 gpurun_out/r05i_tests.log; exit 1; }
tail -1 gpurun_out/r05i_tests.log
timeout -k 10 300 python3 tools/part_breakdown.py 100000000 20 > gpurun_out/r05i_A.txt 2>&1 || { tail -5 gpurun_out/r05i_A.txt; exit 1; }
grep -E "page_merge|merge_count|named|wall" gpurun_out/r05i_A.txt
if [ -f abx/libB.so ]; then
  ST_LIB=abx/libB.so timeout -k 10 300 python3 tools/part_breakdown.py 100000000 20 > gpurun_out/r05i_B.txt 2>&1 || { tail -5 gpurun_out/r05i_B.txt; exit 1; }
  grep -E "page_merge|merge_count|named|wall" gpurun_out/r05i_B.txt
fi
