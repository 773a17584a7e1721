#!/bin/bash
# A/B of k_rehash_fused shapes (ST_RF: 0 = 16 waves x 2 blocks in flight,
# 1 = 8 x 4, 2 = 8 x 6, 3 = 16 x 3): the headline bench line per shape
# (bench.py asserts the top hash after the timed rehashes).
mkdir -p gpurun_out
for cfg in "$@"; do
  ST_RF=$cfg timeout -k 10 240 python3 bench.py --steps 50 --warmup 5 --no-extras --no-pmc --no-cpu > gpurun_out/rf_$cfg.json 2> gpurun_out/rf_$cfg.err || { echo "cfg $cfg failed rc=$?"; tail -5 gpurun_out/rf_$cfg.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/rf_$cfg.json')); print('ST_RF=$cfg', d['value']/1e9, 'Gkeys/s', d['ms_per_step'], 'ms/step', d['roofline']['kernel_avg_ms'], 'ms kernel')"
done
