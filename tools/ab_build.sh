#!/bin/bash
# Headline bench line of another build (ST_LIB=<.so>) next to the in-tree
# build, alternating, on the same box.  Usage: tools/ab_build.sh <so> [reps]
SO=$1; N=${2:-2}
for i in $(seq 1 $N); do
  for lib in "$SO" ""; do
    ST_LIB=$lib timeout -k 10 240 python3 bench.py --steps 50 --warmup 5 --no-extras --no-pmc --no-cpu > gpurun_out/abb.json 2> gpurun_out/abb.err || { echo "failed ($lib)"; tail -5 gpurun_out/abb.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/abb.json')); print('${lib:-in-tree}', round(d['value']/1e9,2), 'Gkeys/s', d['roofline']['kernel_avg_ms'], 'ms kernel')"
  done
done
