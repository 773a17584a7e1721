#!/bin/bash
# A/B of rehash variants (env knobs) in one GPU call; parity first.
R=$(pwd)
timeout -k 10 300 python3 -m pytest $R/tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $R/gpurun_out/ab_tests.log 2>&1 || exit 1
for v in 3 3; do
  ST_K1=$v timeout -k 10 200 python3 $R/bench.py --steps 30 --warmup 5 --no-cpu --no-extras > $R/gpurun_out/ab_k1$v.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('$R/gpurun_out/ab_k1$v.json')); print('k1=$v', d['value']/1e9, d['ms_per_step'], d['roofline']['kernel_avg_ms'])" >> $R/gpurun_out/ab_summary.txt
done
bash $R/tools/trace_short.sh lv3
