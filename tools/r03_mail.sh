#!/bin/bash
# Epoch-stamped mailboxes: fused-rehash parity at every geometry, BASELINE-size
# configs, group time, bench line.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_fused_geometries.py tests/test_gpu_scale.py tests/test_parallel.py tests/test_gpu_parity.py tests/test_term_keys.py tests/test_remote_exchange.py tests/test_exchange_apply.py tests/test_partitioned_exchange.py -x -q --timeout 600 --timeout-method thread -m gpu > gpurun_out/mail_tests.log 2>&1
rc=$?; tail -2 gpurun_out/mail_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/group_time.py 512 1000000 5 > gpurun_out/mail_group.txt 2>&1 || exit $?
tail -1 gpurun_out/mail_group.txt
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-cpu > gpurun_out/mail_bench.json 2> gpurun_out/mail_bench.err || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/mail_bench.json'))
print('head', round(d['value']/1e9,2), d['roofline']['kernel_avg_ms'], 'cmp', d['compare']['ms_per_compare'], d['compare']['kernel_ms_per_compare'], 'ens', d['ensembles']['kernel_ms_per_batch'], d['ensembles']['roofline']['frac'], 'part', d['partition']['ms_per_batch'], d['config1']['per_key_latency_us']['gpu_get'], d['config1']['per_key_latency_us']['gpu_insert'])"
