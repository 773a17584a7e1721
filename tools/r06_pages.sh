# GPU box: paged-stream / ingest tests, then the config-5 breakdown.  Usage: bash tools/r06_pages.sh TAG
set -o pipefail
tag=${1:-x}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_paged_stream.py tests/test_ingest_small_batches.py "tests/test_gpu_scale.py::test_config5_partitioned_streaming_100m" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_ptests.log 2>&1 || { tail -40 gpurun_out/${tag}_ptests.log; exit 1; }
tail -2 gpurun_out/${tag}_ptests.log
timeout -k 10 300 python3 tools/part_breakdown.py 100000000 20 > gpurun_out/${tag}_breakdown.txt 2>&1 || { tail -5 gpurun_out/${tag}_breakdown.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${tag}_breakdown.txt | tail -22
