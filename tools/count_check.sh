# Entry accounting of the paged streaming path (pages_count_check.py), then
# the config-5 breakdown.  Usage: bash tools/count_check.sh TAG
set -o pipefail
tag=${1:-x}
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/pages_count_check.py 40000000 6 check > gpurun_out/${tag}_count_pages.txt 2>&1 || { tail -20 gpurun_out/${tag}_count_pages.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${tag}_count_pages.txt | tail -6
timeout -k 10 300 python3 tools/part_breakdown.py 100000000 20 > gpurun_out/${tag}_breakdown.txt 2>&1 || { tail -5 gpurun_out/${tag}_breakdown.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${tag}_breakdown.txt
