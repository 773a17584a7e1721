#!/bin/bash
# Config-4 / config-5 evidence: fused-kernel phase stamps on one 1M-key tree
# (the config-4 tree), rocprofv3 kernel stats of a 64 x 1M group rehash and of
# the config-5 leg (100M-key tree, 1M-key batches).
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
ST_LEVEL_STAMPS=1 timeout -k 10 120 python3 tools/stamps_1m.py > gpurun_out/stamps_1m.txt 2>&1 || exit $?
grep "fused" gpurun_out/stamps_1m.txt | tail -20
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_group -o run -- python3 $R/tools/group_prof.py 64 > gpurun_out/prof_group.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_part -o run -- python3 $R/tools/part_prof.py > gpurun_out/prof_part.log 2>&1 || exit $?
find gpurun_out/prof_group gpurun_out/prof_part -name "*kernel_stats.csv" | head
