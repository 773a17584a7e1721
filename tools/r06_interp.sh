# GPU box: paged / int64 / ingest tests, then config-5 breakdowns of the build against abx/libNOINT.so.
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_paged_stream.py tests/test_int64_runs.py tests/test_ingest_small_batches.py "tests/test_gpu_scale.py::test_config5_partitioned_streaming_100m" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06aq_tests.log 2>&1 || { tail -30 gpurun_out/r06aq_tests.log; exit 1; }
tail -2 gpurun_out/r06aq_tests.log
bash tools/r06_abn.sh r06aq PROBE && grep -H merge_count gpurun_out/r06aq_bd_*.txt
