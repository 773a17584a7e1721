#!/bin/bash
# Round-3 closing evidence: whole GPU suite, default bench line (PMC, CPU
# baselines, every leg), isolated rocprofv3 trace of the timed rehash.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/f2_suite.log 2>&1
rc=$?; tail -2 gpurun_out/f2_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 bench.py > gpurun_out/f2_bench_full.json 2> gpurun_out/f2_bench_full.err || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/f2_bench_full.json'))
print('head', round(d['value']/1e9,2), d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'], d['roofline']['traffic'], 'cmp', d['compare']['ms_per_compare'], 'ens', d['ensembles']['kernel_ms_per_batch'], d['ensembles']['roofline']['frac'], 'part', d['partition']['ms_per_batch'])"
timeout -k 10 400 bash tools/trace_rehash.sh r03f2 > gpurun_out/trace_r03f2.log 2>&1 || exit $?
grep rehash_fused gpurun_out/trace_r03f2/trace/run_kernel_stats.csv | cut -c1-200
