#!/bin/bash
# Progressive rehash (ST_REHASH=prog): quick parity, stamps on a 10M tree,
# headline A/B against k_rehash_fused, then the whole GPU suite with prog.
mkdir -p gpurun_out
export ST_REHASH=prog
timeout -k 10 240 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/prog_parity.log 2>&1
rc=$?; tail -3 gpurun_out/prog_parity.log; [ $rc -eq 0 ] || exit $rc
ST_LEVEL_STAMPS=1 timeout -k 10 120 python3 tools/stamps.py > gpurun_out/prog_stamps.txt 2>&1 || exit $?
grep -E "stamp" gpurun_out/prog_stamps.txt | tail -16
timeout -k 10 240 python3 bench.py --steps 50 --warmup 5 --no-extras --no-pmc --no-cpu > gpurun_out/prog_head.json 2> gpurun_out/prog_head.err || exit $?
ST_REHASH=fused timeout -k 10 240 python3 bench.py --steps 50 --warmup 5 --no-extras --no-pmc --no-cpu > gpurun_out/fused_head.json 2> gpurun_out/fused_head.err || exit $?
for f in prog fused; do python3 -c "import json,sys; d=json.load(open('gpurun_out/${f}_head.json')); print('$f', round(d['value']/1e9,2), 'Gkeys/s', d['roofline']['kernel_avg_ms'], 'ms kernel')"; done
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_prog.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_prog.log; exit $rc
