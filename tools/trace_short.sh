#!/bin/bash
# Kernel trace of a short rehash-only bench (tag = $1), env passed through.
R=$(pwd); TAG=${1:-x}
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/tr_$TAG -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --no-extras > $R/gpurun_out/tr_$TAG.json 2>/dev/null
