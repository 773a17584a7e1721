#!/bin/bash
# Compare parity tests (term keys included), compare-walk stamps, bench line.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_term_keys.py tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_remote_exchange.py tests/test_exchange_apply.py tests/test_partitioned_exchange.py -x -q --timeout 300 --timeout-method thread -m gpu -k "compare or exchange or diff or config3 or remote or term" > gpurun_out/cmp_tests.log 2>&1
rc=$?; tail -3 gpurun_out/cmp_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/cmp_stamps.py > gpurun_out/cmp_stamps.txt 2>&1 || exit $?
grep -E "stamp (verify|merge|end|staged)|diffs" gpurun_out/cmp_stamps.txt | tail -5
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-cpu > gpurun_out/cmp_bench.json 2> gpurun_out/cmp_bench.err || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/cmp_bench.json'))
print('head', round(d['value']/1e9,2), d['roofline']['kernel_avg_ms'], 'cmp', d['compare']['ms_per_compare'], d['compare']['kernel_ms_per_compare'], 'ens', d['ensembles']['ms_per_batch'], 'part', d['partition']['ms_per_batch'])"
