#!/bin/bash
# GPU suite + config-5 batch breakdown (span merge vs entry walk) + headline.
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_r03.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r03.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/part_breakdown.py > gpurun_out/part_bd_span.txt 2>&1 || exit $?
ST_MERGE=1 timeout -k 10 300 python -u tools/part_breakdown.py > gpurun_out/part_bd_walk.txt 2>&1 || exit $?
tail -3 gpurun_out/part_bd_span.txt; tail -3 gpurun_out/part_bd_walk.txt
ST_LEVEL_STAMPS=1 timeout -k 10 120 python3 tools/stamps_1m.py > gpurun_out/stamps_1m.txt 2>&1 || exit $?
timeout -k 10 240 python3 bench.py --steps 50 --warmup 5 --no-extras --no-pmc --no-cpu > gpurun_out/head.json 2> gpurun_out/head.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/head.json')); print('headline', round(d['value']/1e9,2), 'Gkeys/s', d['roofline']['kernel_avg_ms'], 'ms kernel')"
