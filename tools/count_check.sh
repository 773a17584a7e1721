# Entry accounting of the paged streaming path (pages_count_check.py), then
# the config-5 breakdown.  Usage: bash tools/count_check.sh TAG
set -o pipefail
tag=${1:-x}
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/pages_count_check.py 40000000 6 check > gpurun_out/${tag}_count_pages.txt 2>&1 || { tail -20 gpurun_out/${tag}_count_pages.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${tag}_count_pages.txt | tail -6
timeout -k 10 300 python3 tools/part_breakdown.py 100000000 20 > gpurun_out/${tag}_breakdown.txt 2>&1 || { tail -5 gpurun_out/${tag}_breakdown.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${tag}_breakdown.txt
timeout -k 10 300 python3 tools/repair_breakdown.py 10000000 10 > gpurun_out/${tag}_repair.txt 2>&1 || { tail -20 gpurun_out/${tag}_repair.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${tag}_repair.txt
timeout -k 10 400 python -u -m pytest tests/test_paged_stream.py tests/test_fused_geometries.py tests/test_gpu_parity.py tests/test_small_path.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
