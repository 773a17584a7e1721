#!/bin/bash
# GPU box: the compare's parity tests (default path), the per-key kernel's
# clock stamps, then the staged-pair A/B (tools/ab_cmp_staged.sh).
# Usage: bash tools/compare_checks.sh <tag>
set -o pipefail
TAG=${1:-r04}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_compare_shapes.py tests/test_gpu_parity.py tests/test_exchange_apply.py tests/test_partitioned_exchange.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/${TAG}_cmp_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_cmp_tests.log; [ $rc -eq 0 ] || exit $rc
ST_SMALL_STAMPS=1 timeout -k 10 120 python -u tools/small_stamps.py > gpurun_out/${TAG}_small_stamps.txt 2>&1 || exit 1
bash tools/ab_cmp_staged.sh $TAG
