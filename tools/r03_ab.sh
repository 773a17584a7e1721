#!/bin/bash
# A/B: the build before 6d10aec (ab/lib_d68b395.so) vs the in-tree build, full
# bench line without PMC / CPU legs; then the config-5 merge walk vs span merge.
mkdir -p gpurun_out
for lib in ab/lib_d68b395.so ""; do
  tag=${lib:+old}; tag=${tag:-new}
  ST_LIB=$lib timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-cpu > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || exit $?
done
ST_MERGE=1 timeout -k 10 300 python -u tools/part_breakdown.py > gpurun_out/part_bd_walk.txt 2>&1 || exit $?
tail -3 gpurun_out/part_bd_walk.txt
