#!/bin/bash
# Whole GPU suite, then the bench line without the PMC / CPU legs.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/sb_suite.log 2>&1
rc=$?; tail -2 gpurun_out/sb_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-cpu > gpurun_out/sb_bench.json 2> gpurun_out/sb_bench.err || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/sb_bench.json'))
print('head', round(d['value']/1e9,2), d['roofline']['kernel_avg_ms'], 'cmp', d['compare']['ms_per_compare'], d['compare']['kernel_ms_per_compare'], 'ens', d['ensembles']['ms_per_batch'], d['ensembles']['kernel_ms_per_batch'], d['ensembles']['roofline']['frac'], 'part', d['partition']['ms_per_batch'])"
