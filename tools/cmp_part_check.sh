#!/bin/bash
# GPU box: compare-related parity tests, a compare-only bench line and a
# kernel trace of the config-5 leg.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "compare or exchange or golden or scale" > gpurun_out/pytest_cmp.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_cmp.log; exit 1; }
tail -2 gpurun_out/pytest_cmp.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/part_trace -o run -- python3 tools/part_prof.py > gpurun_out/part.txt 2>&1 || { echo "part trace failed"; tail gpurun_out/part.txt; exit 1; }
tail -2 gpurun_out/part.txt
