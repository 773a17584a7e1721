#!/bin/bash
# GPU box: streaming-delta parity tests, the ingest/per-key/partition suites
# around it, then the config-5 batch breakdown (1M-key batches into 100M keys).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_delta_stream.py tests/test_leveldb_format.py tests/test_term_keys.py tests/test_ingest_small_batches.py tests/test_small_path.py tests/test_exchange_apply.py tests/test_concurrent_trees.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/delta_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|Error|assert" gpurun_out/delta_tests.log | tail -25; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/part_breakdown.py 100000000 30 delta > gpurun_out/delta_breakdown.txt 2>&1 || { tail -20 gpurun_out/delta_breakdown.txt; exit 1; }
cat gpurun_out/delta_breakdown.txt
