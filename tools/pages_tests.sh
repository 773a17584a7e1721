set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_paged_stream.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r05c_pages_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|Error|assert|page check" gpurun_out/r05c_pages_tests.log | tail -30; exit $rc
