#!/bin/bash
# Compact level-H messages (3 windows per CU for sparse groups) + new compare
# gather: focused parity, full bench line, then the whole GPU suite.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fused_geometries.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/v2_tests.log 2>&1
rc=$?; tail -2 gpurun_out/v2_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-cpu > gpurun_out/v2_bench.json 2> gpurun_out/v2_bench.err || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/v2_bench.json'))
print('head', round(d['value']/1e9,2), d['roofline']['kernel_avg_ms'], 'cmp', d['compare']['ms_per_compare'], d['compare']['kernel_ms_per_compare'], 'ens', d['ensembles']['ms_per_batch'], d['ensembles']['kernel_ms_per_batch'], d['ensembles']['roofline']['frac'], 'part', d['partition']['ms_per_batch'])"
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/v2_suite.log 2>&1
rc=$?; tail -2 gpurun_out/v2_suite.log; exit $rc
