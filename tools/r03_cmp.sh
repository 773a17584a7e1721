#!/bin/bash
# Compare: parity tests, per-wave stamps, bench compare leg.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_remote_exchange.py tests/test_exchange_apply.py tests/test_partitioned_exchange.py -x -q --timeout 300 --timeout-method thread -m gpu -k "compare or exchange or diff or config3 or remote" > gpurun_out/cmp_tests.log 2>&1
rc=$?; tail -2 gpurun_out/cmp_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/cmp_stamps.py > gpurun_out/cmp_stamps.txt 2>&1 || exit $?
tail -12 gpurun_out/cmp_stamps.txt
