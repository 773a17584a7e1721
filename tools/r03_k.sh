#!/bin/bash
# Compare stamps (finer flush phases), config-5 batch breakdown, GPU suite.
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/cmp_stamps.py > gpurun_out/cmp_stamps2.txt 2>&1 || exit $?
grep -E "stamp (children|flush|inner|values|staged|verify|merge|end)" gpurun_out/cmp_stamps2.txt | tail -8
timeout -k 10 300 python -u tools/part_breakdown.py > gpurun_out/part_bd_k.txt 2>&1 || exit $?
grep -E "verify|segment_hash|wall" gpurun_out/part_bd_k.txt
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/k_suite.log 2>&1
rc=$?; tail -2 gpurun_out/k_suite.log; exit $rc
