#!/bin/bash
# GPU-box: parity + smoke + default bench, then A/B of the fused vs v3 rehash.
set -o pipefail
R=$(pwd)
bash $R/tools/round_check.sh || exit 1
for f in 2 0 1 2; do
  ST_REHASH=$f timeout -k 10 200 python3 $R/bench.py --steps 30 --warmup 5 --no-cpu --no-extras > $R/gpurun_out/ab_f$f.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('$R/gpurun_out/ab_f$f.json')); print('mode=$f', d['value']/1e9, d['ms_per_step'])" | tee -a $R/gpurun_out/ab_summary.txt
done
