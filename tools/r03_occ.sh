#!/bin/bash
# Group rehash at 6 waves per SIMD (three sparse windows per CU): parity, time.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fused_geometries.py tests/test_gpu_scale.py tests/test_parallel.py -x -q --timeout 300 --timeout-method thread -m gpu -k "group or ensemble or config4 or geometry or empty" > gpurun_out/occ_tests.log 2>&1
rc=$?; tail -2 gpurun_out/occ_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/group_time.py 512 1000000 5 > gpurun_out/occ_group.txt 2>&1 || exit $?
tail -3 gpurun_out/occ_group.txt
