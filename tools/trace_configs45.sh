#!/bin/bash
# rocprofv3 kernel stats of the config-4 group rehash (512 trees x 1M keys,
# 5 timed st_rehash_group launches: tools/group_time.py) and of config-5
# write batches (1M keys into a 100M-key tree: tools/part_breakdown.py).
# Usage (on the box, from the repo root): bash tools/trace_configs45.sh <tag>
set -euo pipefail
TAG=${1:-r04}
R=$(pwd)
OUT=$R/gpurun_out/trace45_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/group -o run -- python3 $R/tools/group_time.py 512 1000000 5 > $OUT/group.txt 2> $OUT/group.err
cat $OUT/group.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/config5 -o run -- python3 $R/tools/part_breakdown.py 100000000 30 > $OUT/config5.txt 2> $OUT/config5.err
cat $OUT/config5.txt
