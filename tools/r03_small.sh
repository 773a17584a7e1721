#!/bin/bash
# Small (per-key) path: parity tests, per-key latency, stamps.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_small_path.py tests/test_gpu_parity.py tests/test_term_keys.py tests/test_concurrent_trees.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/small_tests.log 2>&1
rc=$?; tail -2 gpurun_out/small_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/perkey_lat.py 2000 > gpurun_out/perkey.txt 2>&1 || exit $?
tail -4 gpurun_out/perkey.txt
timeout -k 10 300 python -u tools/small_stamps.py > gpurun_out/small_stamps.txt 2>&1 || exit $?
grep -c "op=0" gpurun_out/small_stamps.txt
