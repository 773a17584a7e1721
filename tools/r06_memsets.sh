# GPU box: paged + ingest + int64 tests, then the config-5 breakdown (fused memsets).  Usage: bash tools/r06_memsets.sh TAG
set -o pipefail
tag=${1:-x}
timeout -k 10 600 python -u -m pytest tests/test_paged_stream.py tests/test_int64_runs.py tests/test_ingest_small_batches.py tests/test_gpu_parity.py tests/test_stream_order.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
bash tools/r06_abn.sh $tag
