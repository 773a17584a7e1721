#!/bin/bash
# GPU-box A/B of env knobs: parity tests once, then one bench line per setting.
# Usage: bash tools/ab_env.sh "ST_LEVELS=1" "ST_LEVELS=0" ...
set -o pipefail
R=$(pwd)
mkdir -p $R/gpurun_out
timeout -k 10 400 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/ab_tests.log 2>&1 || { tail -30 $R/gpurun_out/ab_tests.log; exit 1; }
tail -2 $R/gpurun_out/ab_tests.log
i=0
for kv in "$@"; do
  i=$((i+1))
  env $kv timeout -k 10 200 python3 $R/bench.py --steps 30 --warmup 5 --no-cpu --no-extras > $R/gpurun_out/ab_$i.json 2>$R/gpurun_out/ab_$i.err || { tail $R/gpurun_out/ab_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$R/gpurun_out/ab_$i.json')); r=d['roofline']; print('$kv', round(d['value']/1e9,2), 'G keys/s', d['ms_per_step'], 'ms; K1', r['kernel_avg_ms'], 'levels', r['level_rehash_avg_ms_per_step'])"
done
