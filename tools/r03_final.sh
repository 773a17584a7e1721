#!/bin/bash
# Round-3 evidence: the default bench line (PMC traffic, CPU baselines, every
# leg) and an isolated rocprofv3 trace of the timed rehash loop.
mkdir -p gpurun_out
timeout -k 10 900 python3 bench.py > gpurun_out/r03_bench_full.json 2> gpurun_out/r03_bench_full.err || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/r03_bench_full.json'))
print('head', round(d['value']/1e9,2), d['roofline']['kernel_avg_ms'], d['roofline']['frac'], d['roofline']['traffic'], 'cmp', d['compare']['ms_per_compare'], 'ens', d['ensembles']['ms_per_batch'], d['ensembles'].get('roofline',{}).get('frac'), 'part', d['partition']['ms_per_batch'])"
timeout -k 10 400 bash tools/trace_rehash.sh r03 > gpurun_out/trace_r03.log 2>&1 || exit $?
tail -2 gpurun_out/trace_r03.log
