#!/bin/bash
# Isolated kernel trace of ONLY the timed 10M-key rehash loop (bench.py
# --no-extras --no-cpu), so the K1/K2 means in profiles/ come from the same
# launches bench.py times.  Usage (on the box): bash tools/trace_rehash.sh <tag>
set -euo pipefail
TAG=${1:-r02}
R=$(pwd)
OUT=$R/gpurun_out/trace_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 $R/bench.py --steps 50 --warmup 5 --no-cpu --no-extras --no-cold --no-pmc > $OUT/bench.json 2> $OUT/bench.err
echo "trace done"
cat $OUT/bench.json
