#!/bin/bash
# GPU box: the paged-layout parity tests and the ingest / per-key / exchange
# suites, then config-5 breakdowns with the pages on and off.
# Usage: bash tools/check_pages.sh <tag>
set -o pipefail
TAG=${1:-r05}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_paged_stream.py tests/test_ingest_small_batches.py tests/test_small_path.py tests/test_exchange_apply.py tests/test_concurrent_trees.py tests/test_term_keys.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pages_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|Error|assert" gpurun_out/${TAG}_pages_tests.log | tail -30; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/part_breakdown.py 100000000 20 > gpurun_out/${TAG}_config5_breakdown_pages.txt 2>&1 || { tail -20 gpurun_out/${TAG}_config5_breakdown_pages.txt; exit 1; }
cat gpurun_out/${TAG}_config5_breakdown_pages.txt
timeout -k 10 300 python3 tools/part_breakdown.py 100000000 10 csr > gpurun_out/${TAG}_config5_breakdown_csr.txt 2>&1 || { tail -20 gpurun_out/${TAG}_config5_breakdown_csr.txt; exit 1; }
tail -3 gpurun_out/${TAG}_config5_breakdown_csr.txt
