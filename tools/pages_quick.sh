#!/bin/bash
# GPU box: the paged-layout parity tests (checked build), then a config-5
# breakdown with the pages on.  Usage: bash tools/pages_quick.sh <tag>
set -o pipefail
TAG=${1:-r05}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_paged_stream.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pages_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|Error|assert|page check" gpurun_out/${TAG}_pages_tests.log | tail -30; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/part_breakdown.py 100000000 20 > gpurun_out/${TAG}_config5_breakdown_pages.txt 2>&1 || { tail -20 gpurun_out/${TAG}_config5_breakdown_pages.txt; exit 1; }
cat gpurun_out/${TAG}_config5_breakdown_pages.txt
