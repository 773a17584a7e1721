#!/bin/bash
# Ingest merge with per-workgroup staged segment data: ingest parity tests,
# config-5 batch breakdown, then the whole GPU suite.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ingest_small_batches.py tests/test_gpu_parity.py tests/test_small_path.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/merge_tests.log 2>&1
rc=$?; tail -2 gpurun_out/merge_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/part_breakdown.py > gpurun_out/part_bd_staged.txt 2>&1 || exit $?
grep -E "merge|wall" gpurun_out/part_bd_staged.txt
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/merge_suite.log 2>&1
rc=$?; tail -2 gpurun_out/merge_suite.log; exit $rc
