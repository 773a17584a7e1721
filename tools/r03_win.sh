#!/bin/bash
# Packed-message fused rehash: GPU suite, full bench line, phase stamps (10M / 1M).
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/win_parity.log 2>&1
rc=$?; tail -2 gpurun_out/win_parity.log; [ $rc -eq 0 ] || exit $rc
ST_LEVEL_STAMPS=1 timeout -k 10 120 python3 tools/stamps.py > gpurun_out/win_stamps.txt 2>&1 || exit $?
ST_LEVEL_STAMPS=1 timeout -k 10 120 python3 tools/stamps_1m.py > gpurun_out/win_stamps_1m.txt 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-cpu > gpurun_out/win.json 2> gpurun_out/win.err || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/win.json'))
print('head', round(d['value']/1e9,2), d['roofline']['kernel_avg_ms'], 'cmp', d['compare']['ms_per_compare'], 'ens', d['ensembles']['ms_per_batch'], 'part', d['partition']['ms_per_batch'], 'repair', d['repair']['ms_per_repair'])"
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_win.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_win.log; exit $rc
