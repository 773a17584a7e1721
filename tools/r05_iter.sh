# Paged-stream + ingest GPU tests, then the config-5 breakdown.  Usage: bash tools/r05_iter.sh TAG
set -o pipefail
tag=${1:-x}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_paged_stream.py tests/test_ingest_small_batches.py tests/test_concurrent_trees.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
timeout -k 10 300 python3 tools/part_breakdown.py 100000000 20 > gpurun_out/${tag}_breakdown.txt 2>&1 || { tail -5 gpurun_out/${tag}_breakdown.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${tag}_breakdown.txt
