# Paged / small / compare tests on the in-tree build, then page-merge occupancy variants.
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_paged_stream.py tests/test_small_path.py tests/test_compare_shapes.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/abc_tests.log 2>&1 || { tail -30 gpurun_out/abc_tests.log; exit 1; }
tail -1 gpurun_out/abc_tests.log
timeout -k 10 300 python3 tools/part_breakdown.py 100000000 20 > gpurun_out/abc_A.txt 2>&1 || exit 1
echo "== default"; grep -E "page_merge|timing off" gpurun_out/abc_A.txt
for v in MK8 VC8; do
  ST_LIB=abx/lib$v.so timeout -k 10 300 python3 tools/part_breakdown.py 100000000 20 > gpurun_out/abc_$v.txt 2>&1 || exit 1
  echo "== $v"; grep -E "page_merge|timing off" gpurun_out/abc_$v.txt
done
